"""Summaries of a rocprofv3 database (rocpd .db): per-kernel stats and the
timeline of the last N dispatches.  python tools/prof_db.py DIR [N]"""
import glob
import sqlite3
import sys


def main():
    d = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    for db in glob.glob(d + '/**/*.db', recursive=True):
        c = sqlite3.connect(db)
        print('# kernel stats (ns):', db)
        for name, cnt, avg, mn, mx in c.execute(
                "select name, count(*), avg(duration), min(duration), max(duration) from kernels "
                "group by name order by sum(duration) desc"):
            print('%-60s %6d %12.0f %12.0f %12.0f' % (name.split('(')[0][:60], cnt, avg, mn, mx))
        if n:
            rows = list(c.execute("select name, stream_id, start, end from kernels order by start"))[-n:]
            t0 = rows[0][2]
            print('# timeline (us from first shown): stream start end dur name')
            for name, st, a, b in rows:
                print('%3s %10.1f %10.1f %8.1f %s' % (st, (a - t0) / 1e3, (b - t0) / 1e3, (b - a) / 1e3,
                                                     name.split('(')[0][:50]))


if __name__ == '__main__':
    main()

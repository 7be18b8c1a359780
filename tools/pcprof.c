/* Minimal sampling profiler for the library's host code (CPU container only):
 * SIGPROF every 1/hz CPU-second of the process, the interrupted PC counted
 * in a table; pcprof_stop(path) writes "count library offset" lines (dladdr)
 * for tools/pcprof.py to resolve with addr2line.
 *   gcc -O2 -shared -fPIC tools/pcprof.c -o tools/pcprof.so -ldl
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/time.h>
#include <ucontext.h>

#define NB (1 << 20)
static uint64_t pcs[NB];
static uint32_t cnt[NB];
static volatile uint64_t dropped;

static void on_prof(int sig, siginfo_t* si, void* uc_) {
  (void)sig;
  (void)si;
  ucontext_t* uc = (ucontext_t*)uc_;
  uint64_t pc = (uint64_t)uc->uc_mcontext.gregs[REG_RIP];
  uint64_t h = (pc * 0x9E3779B97F4A7C15ull) >> 44;
  for (int i = 0; i < 64; ++i, h = (h + 1) & (NB - 1)) {
    uint64_t cur = __atomic_load_n(&pcs[h], __ATOMIC_RELAXED);
    if (cur == pc) {
      __atomic_fetch_add(&cnt[h], 1, __ATOMIC_RELAXED);
      return;
    }
    if (cur == 0) {
      uint64_t z = 0;
      if (__atomic_compare_exchange_n(&pcs[h], &z, pc, 0, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
        __atomic_fetch_add(&cnt[h], 1, __ATOMIC_RELAXED);
        return;
      }
      if (z == pc) {
        __atomic_fetch_add(&cnt[h], 1, __ATOMIC_RELAXED);
        return;
      }
    }
  }
  __atomic_fetch_add(&dropped, 1, __ATOMIC_RELAXED);
}

int pcprof_start(int hz) {
  memset(pcs, 0, sizeof pcs);
  memset(cnt, 0, sizeof cnt);
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  if (sigaction(SIGPROF, &sa, NULL)) return -1;
  struct itimerval it;
  it.it_interval.tv_sec = 0;
  it.it_interval.tv_usec = 1000000 / (hz > 0 ? hz : 1000);
  it.it_value = it.it_interval;
  return setitimer(ITIMER_PROF, &it, NULL);
}

int pcprof_stop(const char* path) {
  struct itimerval it;
  memset(&it, 0, sizeof it);
  setitimer(ITIMER_PROF, &it, NULL);
  signal(SIGPROF, SIG_IGN);
  FILE* f = fopen(path, "w");
  if (!f) return -1;
  for (int i = 0; i < NB; ++i) {
    if (!pcs[i]) continue;
    Dl_info di;
    if (dladdr((void*)pcs[i], &di) && di.dli_fname)
      fprintf(f, "%u %s 0x%llx\n", cnt[i], di.dli_fname,
              (unsigned long long)(pcs[i] - (uint64_t)di.dli_fbase));
    else
      fprintf(f, "%u ? 0x%llx\n", cnt[i], (unsigned long long)pcs[i]);
  }
  fprintf(f, "%llu dropped 0x0\n", (unsigned long long)dropped);
  fclose(f);
  return 0;
}

#!/usr/bin/env python3
"""Single-rank RCCL gather check in the two library load orders a process can
have: liblt first (bench.py), or PyTorch first (liblt then binds torch's
bundled HIP runtime and must use torch's RCCL).  Prints the RCCL in use.

    python tools/gather_check.py [--torch-first]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if '--torch-first' in sys.argv:
    import torch  # noqa: F401
from lattice_based_tagger_amd import _capi, synth  # noqa: E402
lib = _capi.load()
if '--torch-first' not in sys.argv:
    import torch  # noqa: F401,E402
import numpy as np  # noqa: E402
from oracle import lt_oracle  # noqa: E402

raw = synth.make_lattices(200, seed=3, eojeols=8)
sm = synth.make_model(raw, seed=3, n_features=10_000)
packed, keys, coefs = synth.pack_fast(raw, sm)
ctx = _capi.Context(0)
dm = _capi.DeviceModel(ctx, keys, coefs)
db = _capi.DeviceBatch(ctx, packed, max_k=5)
comm = _capi.Comm(ctx, 1, 0, _capi.comm_unique_id())
comm.prepare(db, 5)
db.launch(dm, 5)
comm.launch(db)
comm.sync()
comm.fetch()
ctx.sync()
got = comm.view(0)
exp = lt_oracle.decode(packed, keys, coefs, 5)
ok = (np.array_equal(got[0], exp[0]) and np.array_equal(got[1], exp[1])
      and np.array_equal(got[2].view(np.uint64), exp[2].view(np.uint64)) and np.array_equal(got[3], exp[3]))
print('gather_check', 'torch-first' if '--torch-first' in sys.argv else 'liblt-first',
      lib.lt_comm_library().decode(), 'OK' if ok else 'MISMATCH')
comm.close(); db.close(); dm.close(); ctx.close()
sys.exit(0 if ok else 1)

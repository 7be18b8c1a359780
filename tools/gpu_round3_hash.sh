# A/B of the one-mix power-of-two slot hash (HASH_VERSION 4, "hash") against
# the previous build ("base"), a timing-only build without the 8-9 term sum
# path ("no9", wrong for those expansions: never a product build), the
# parity suites on the new default library, then the Tagger e2e diagnostics.
set -o pipefail
KS="5 1 16 2" LIBS="base hash no9 base hash" bash tools/gpu_ab.sh || exit 1
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plugins.py tests/test_gpu_api.py tests/test_modelpack.py tests/test_gpu_tagger.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_hash.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_hash.log; exit 1; }
tail -1 gpurun_out/pytest_hash.log
bash tools/gpu_round3_e2e3.sh

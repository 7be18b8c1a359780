# A/B of the one-mix power-of-two slot hash (HASH_VERSION 4) against the
# previous build, then the parity suites on the new default library.
set -o pipefail
KS="1 5 16 2" LIBS="base hash base hash" bash tools/gpu_ab.sh || exit 1
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plugins.py tests/test_gpu_api.py tests/test_modelpack.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_hash.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_hash.log; exit 1; }
tail -1 gpurun_out/pytest_hash.log
PROFILE=1 bash tools/gpu_tagger_e2e.sh

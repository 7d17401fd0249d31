set -u
mkdir -p gpurun_out/r02_t1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02_t1/pytest_gpu.log 2>&1
rc=$?; tail -30 gpurun_out/r02_t1/pytest_gpu.log; echo "pytest rc=$rc"; exit $rc

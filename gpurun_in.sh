set -u
mkdir -p gpurun_out/r01j
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r01j/pytest.log 2>&1; rc=$?; tail -30 gpurun_out/r01j/pytest.log; echo "pytest rc=$rc"

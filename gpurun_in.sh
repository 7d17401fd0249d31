set -u
mkdir -p gpurun_out/r01m
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r01m/pytest.log 2>&1; rc=$?; tail -25 gpurun_out/r01m/pytest.log; echo "pytest rc=$rc"

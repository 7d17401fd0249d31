set -u
mkdir -p gpurun_out/r01l
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r01l/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r01l/pytest.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python scripts/kbench.py --variants 0:0,4:0,1:0,5:0 --workloads c3,c2,c4 --rounds 3 2>&1 | grep -v amdgpu.ids

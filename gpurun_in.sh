set -u
timeout -k 10 300 python -m pytest tests/test_gpu_payload.py tests/test_c1_plumbing.py -x -q 2>&1 | tail -5 &&
timeout -k 10 300 python scripts/pgbench.py --variants 0,1,5,6,7 2>&1 | grep -v amdgpu.ids

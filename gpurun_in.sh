set -u
O=$PWD/dpdk-tcpipstack_amd/rxg/librxg_old.so
timeout -k 10 300 python -m pytest tests -m gpu -x -q 2>&1 | tail -3 &&
timeout -k 10 500 python scripts/kbench.py --variants 0:0::$O,0:0,0:1024,0:1152 --workloads c3,c4,c2 --rounds 4 2>&1 | grep -v amdgpu.ids

set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/txpmc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c --kernel-include-regex "rx_kernel<0" -d gpurun_out/txpmc/$c -o run --output-format csv -- python3 scripts/txbench.py --workloads c3 --rounds 1 --iters 4 > gpurun_out/txpmc/$c.log 2>&1 || exit $?
done

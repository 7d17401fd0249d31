# SQ issue / wait breakdown of the all-small path: C2 as 16 strided bursts per launch, and single launches
set -u
export TMPDIR=/tmp
for W in c2multis c2s; do
  K="rx_kernel<8,"
  O=gpurun_out/r04k/$W; mkdir -p $O
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "$K" -d $O/p1 -o run --output-format csv -- python3 scripts/profrun.py --workload $W --iters 5 --rec 8 > $O/log 2>&1 || { echo "STOP $W"; tail -5 $O/log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR --kernel-include-regex "$K" -d $O/p2 -o run --output-format csv -- python3 scripts/profrun.py --workload $W --iters 5 --rec 8 > $O/log2 2>&1 || { echo "STOP2 $W"; tail -5 $O/log2; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-include-regex "$K" -d $O/p3 -o run --output-format csv -- python3 scripts/profrun.py --workload $W --iters 5 --rec 8 > $O/log3 2>&1 || { echo "STOP3 $W"; tail -5 $O/log3; }
  echo "$W ok"
done

# SQ issue / wait breakdown: the rx kernel (C3, REC8) against the tx kernel over the same batch
set -u
export TMPDIR=/tmp
for W in c3 tx3; do
  case $W in tx3) K="rx_kernel<0," ;; *) K="rx_kernel<8," ;; esac
  O=gpurun_out/r04f/$W; mkdir -p $O
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "$K" -d $O/p1 -o run --output-format csv -- python3 scripts/profrun.py --workload $W --iters 5 --rec 8 > $O/log 2>&1 || { echo "STOP $W"; tail -5 $O/log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR --kernel-include-regex "$K" -d $O/p2 -o run --output-format csv -- python3 scripts/profrun.py --workload $W --iters 5 --rec 8 > $O/log2 2>&1 || { echo "STOP2 $W"; tail -5 $O/log2; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum --kernel-include-regex "$K" -d $O/p3 -o run --output-format csv -- python3 scripts/profrun.py --workload $W --iters 5 --rec 8 > $O/log3 2>&1 || { echo "STOP3 $W"; tail -5 $O/log3; }
  echo "$W ok"
done

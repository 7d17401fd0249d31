#!/bin/bash
# r05zb: the deferred replay corrections' paths (rxg_counters_dev after rxg_sync, a reset
# before the next burst, the next burst's patch launch carrying them) and the replay suites.
set -u
O=gpurun_out/r05zb; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_replay.py tests/test_gpu_fuzz.py tests/test_gpu_multiburst.py tests/test_gpu_group.py > $O/pytest.log 2>&1 || { echo "STOP pytest"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
echo r05zb done

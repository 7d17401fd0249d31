#!/bin/bash
# r05t: the fused forms profiled as their own kernels (PAY 1 copy / 2 by reference): kernel
# trace + FETCH_SIZE / WRITE_SIZE passes over C3.
set -u
export TMPDIR=/tmp
REC=8 bash scripts/gpu_prof.sh r05t pr3 pf3 || exit 1
echo r05t done

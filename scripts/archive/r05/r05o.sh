#!/bin/bash
# r05o: the headline and C2 / C4 legs re-profiled on this round's tree (kernel trace + stats,
# FETCH_SIZE and WRITE_SIZE passes), so every leg's traffic file is from profiles/r05.
set -u
export TMPDIR=/tmp
REC=8 bash scripts/gpu_prof.sh r05o c3 c2 c4 c2multi c2s c2multis || exit 1
echo r05o done

"""TEST INFRASTRUCTURE ONLY — one CPU replica of the faithful oracle, for bench.py's
multi-core cpu_baseline (SURVEY.md §8(d) "one independent replica per host core, disjoint
packet ranges, private tables").  Each replica is its own process, so its ARP list and
tables are private.

    python oracle/replica.py SAMPLE.npz START STOP SECONDS OPT

prints one JSON line {"frames", "bytes", "seconds", "arp_entries"}: frames [START, STOP) of
the sample re-run for SECONDS after one untimed pass over the WHOLE sample, so the replica's
ARP list holds every source the 1-core leg's does (ip.c:26-32 / arp.c:263-280 walk that list
per packet: a shorter list would make each replica faster than the 1-core leg)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402


def main():
    path, s0, s1, seconds, opt = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4]), sys.argv[5]
    z = np.load(path)  # our own file, plain arrays (allow_pickle stays False)
    arena, tcb, live = z["arena"], z["tcb"], z["live"]
    off, lens = z["off"][s0:s1], z["lens"][s0:s1]
    oracle.arp_reset()
    oracle.rx_batch(arena, z["off"], z["lens"], tcb, live, faithful=True, opt=opt)  # learn every source
    frames = nbytes = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        oracle.rx_batch(arena, off, lens, tcb, live, faithful=True, opt=opt)
        frames += len(lens)
        nbytes += int(lens.astype(np.uint64).sum())
    print(json.dumps({"frames": frames, "bytes": nbytes, "seconds": time.perf_counter() - t0,
                      "arp_entries": oracle.arp_count(opt)}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-launch HBM traffic of the rx kernel from rocprofv3 PMC passes (run separately:
--pmc FETCH_SIZE and --pmc WRITE_SIZE, each with only --kernel-include-regex).

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane) coalesced streaming read,
so it is doubled; WRITE_SIZE is exact for 16 B/lane stores and for atomics.

  python scripts/pmc_traffic.py <fetch_csv> <write_csv> <kernel-substring> <out.json> [note]
         [--prov build_fetch.json build_write.json ...]

--prov: the build provenance each counted run wrote (scripts/profrun.py --prov).  They must
name one src= hash; it is stamped into out.json ("build", "source_hash"), which bench.py
compares with the library it loaded (roofline.traffic_matches_build).
"""
import csv
import json
import statistics
import sys


def src_of(build: str):
    """The src= hash of an rxg_build_info() string, or None."""
    return next((w[4:] for w in (build or "").split() if w.startswith("src=")), None)


def stamp(prov_files):
    """The one build the counted runs loaded: {"build", "source_hash"}; ValueError if they differ."""
    builds = [json.load(open(p))["build"] for p in prov_files]
    srcs = {src_of(b) for b in builds}
    if len(srcs) != 1 or None in srcs:
        raise ValueError(f"counted runs loaded different or unstamped builds: {sorted(map(str, srcs))}")
    return {"build": builds[0], "source_hash": srcs.pop()}


def per_launch(path, kernel):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"]]
    return vals


def main():
    argv = sys.argv[1:]
    prov = []
    if "--prov" in argv:
        k = argv.index("--prov")
        argv, prov = argv[:k], argv[k + 1:]
    fetch_csv, write_csv, kernel, out = argv[:4]
    note = argv[4] if len(argv) > 4 else ""
    f = per_launch(fetch_csv, kernel)
    w = per_launch(write_csv, kernel)
    read_b = 2.0 * statistics.median(f) * 1024.0
    write_b = statistics.median(w) * 1024.0
    res = {"kernel": kernel, "launches": [len(f), len(w)],
           "fetch_size_kib_median": statistics.median(f), "write_size_kib_median": statistics.median(w),
           "hbm_read_bytes_per_launch": read_b, "hbm_write_bytes_per_launch": write_b,
           "hbm_bytes_per_launch": read_b + write_b,
           "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count of 16 B/lane streams); "
                         "write = WRITE_SIZE x 1024", "note": note}
    if prov:
        res.update(stamp(prov))
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

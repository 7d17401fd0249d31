"""bench.py's own launcher: `python bench.py --gpus N`
with no launcher around it starts N rank processes itself, and the line reports how many
ranks the collectives saw.  Here (no GPU) through the rehearsal mode: the same spawn, the
same rendezvous and gloo collectives, no measurement."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                            "MASTER_ADDR", "MASTER_PORT")}
    env["HIP_VISIBLE_DEVICES"] = env.get("HIP_VISIBLE_DEVICES", "")
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _lines(out):
    return [json.loads(s) for s in out.splitlines() if s.startswith("{")]


@pytest.mark.parametrize("n", [2, 4])
def test_gpus_n_spawns_n_ranks(n):
    r = _run(["--gpus", str(n), "--no-legs", "--no-cpu"], {"RXG_BENCH_REHEARSE": "1"})
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    line = lines[0]
    assert line["n_gpus"] == n and line["ranks"] == n
    assert sorted(d["rank"] for d in line["devices"]) == list(range(n))
    assert line["max_over_ranks_check"] == float(n)  # the gloo all-reduce saw every rank


def test_gpus_1_is_one_process():
    r = _run(["--gpus", "1", "--no-legs", "--no-cpu"], {"RXG_BENCH_REHEARSE": "1"})
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = _lines(r.stdout)
    assert line["n_gpus"] == 1 and line["ranks"] == 1 and len(line["devices"]) == 1


def test_world_size_disagreeing_with_gpus_fails():
    r = _run(["--gpus", "4"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_more_gpus_than_visible_fails_without_rehearsal():
    r = _run(["--gpus", "2"])
    assert r.returncode != 0 and "GPU(s) visible" in r.stderr


def test_pg_flag_runs_collectives_at_world_1():
    """--pg gloo|nccl initialises a process group even at WORLD_SIZE 1 (VERDICT r4 item 1:
    the RCCL path runs on one GPU before any N > 1 run), with the explicit timeout; here
    through gloo, the rehearsal's CPU backend.  The default (--pg auto) stays group-free."""
    r = _run(["--gpus", "1", "--no-legs", "--no-cpu", "--pg", "gloo", "--pg-timeout", "60"],
             {"RXG_BENCH_REHEARSE": "1"})
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = _lines(r.stdout)
    assert line["collective_backend"] == "gloo" and line["ranks"] == 1
    assert line["max_over_ranks_check"] == 1.0
    r = _run(["--gpus", "1", "--no-legs", "--no-cpu"], {"RXG_BENCH_REHEARSE": "1"})
    (line,) = _lines(r.stdout)
    assert line["collective_backend"] is None


def test_pg_backend_choice():
    import sys
    sys.path.insert(0, ROOT)
    import bench
    assert bench.pg_backend("auto", 1, False) is None
    assert bench.pg_backend("auto", 8, False) == "nccl"
    assert bench.pg_backend("auto", 2, True) == "gloo"
    assert bench.pg_backend("nccl", 1, False) == "nccl"
    assert bench.SOLO_BUDGET_S < 900.0 / 3  # the solo legs end well inside the default timeout


def test_traffic_provenance_reports_a_mismatched_build(tmp_path):
    """roofline.traffic names the build its PMC passes counted
    (scripts/pmc_traffic.py --prov stamps the src= hash), and the line says whether that is
    the library it measured.  A file from another build, or an unstamped one, reports
    traffic_matches_build false."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import bench
    import pmc_traffic
    built = "rxg src=0123456789abcdef rev=abc built=x gfx950"
    for name, stamped, ok in [("same", "0123456789abcdef", True), ("other", "fedcba9876543210", False),
                              ("unstamped", None, False)]:
        tf = tmp_path / f"{name}.json"
        d = {"hbm_bytes_per_launch": 1.0}
        if stamped:
            d["source_hash"] = stamped
        tf.write_text(json.dumps(d))
        p = bench.traffic_provenance(str(tf), built)
        assert p["traffic_matches_build"] is ok and p["traffic_src"] == stamped and p["build_src"] == "0123456789abcdef"
    assert bench.traffic_provenance(None, built)["traffic_matches_build"] is False
    # the stamp: one build across the counted runs, else refused
    a, b = tmp_path / "a.json", tmp_path / "b.json"
    a.write_text(json.dumps({"build": built}))
    b.write_text(json.dumps({"build": built.replace("0123", "9999")}))
    assert pmc_traffic.stamp([str(a), str(a)]) == {"build": built, "source_hash": "0123456789abcdef"}
    with pytest.raises(ValueError):
        pmc_traffic.stamp([str(a), str(b)])


def test_cpu_baseline_host_and_replicas(monkeypatch):
    """the CPU baseline states its host (model, nproc, affinity, quota) and
    runs one replica per usable core, each after learning the WHOLE sample's sources, so every
    replica walks the same ARP list as the 1-core leg (ip.c:26-32, arp.c:263-280)."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import bench
    import oracle
    import pktgen
    import rxg
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    h = bench.host_cpus()
    assert h["nproc"] >= 1 and h["affinity"] >= 1 and h["model"] is not None
    if h["cgroup_quota_cpus"] is None:
        assert h["usable"] == min(3, h["affinity"]) and "OMP_NUM_THREADS" in h["usable_from"]
    else:
        assert h["usable"] <= max(1, int(h["cgroup_quota_cpus"]))
    # 40 sources spread over 400 frames: a replica's own quarter of the range holds only part
    # of them, the whole sample all 40
    nflows = 40
    frames = [pktgen.frame(src_ip=pktgen.ip4(10, 1, 0, f), dst_ip=pktgen.ip4(192, 168, 78, 2), sport=1024 + f,
                           dport=80, flags=0x10, payload=bytes(100)) for f in [i // 10 for i in range(400)]]
    arena, off, lens = pktgen.pack_arena(frames)
    tcb, live = rxg.synthetic_tcb_table(nflows)
    oracle.arp_reset()
    oracle.rx_batch(arena, off, lens, tcb, live, faithful=True, opt="O0")
    assert oracle.arp_count("O0") == nflows
    oracle.arp_reset()
    r = bench.cpu_replicas(arena, off, lens, tcb, live, 4, 0.3)
    assert r is not None and r["cores"] == 4 and r["arp_entries"] == nflows and r["mpps"] > 0

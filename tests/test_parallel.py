"""CPU: the N>1 path (gloo, world_size 2).

* stripe partitioning: encoding each 64-byte-aligned column stripe separately
  and concatenating gives exactly the full-shard parity (the property that
  makes config C4's strong scaling exchange-free), checked with the oracle;
* the max-over-ranks timing reduction and the whole-job throughput formula
  bench.py uses, run in two real processes over gloo.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from bfrs import parallel


def test_stripe_ranges_cover_and_align():
    for S in (64, 128, 33554432, 33554432 + 38, 1000):
        for G in (1, 2, 3, 4, 8):
            r = parallel.stripe_ranges(S, G)
            assert r[0][0] == 0 and r[-1][1] == S
            for (a, b), (c, d) in zip(r, r[1:]):
                assert b == c and a % 64 == 0 and b % 64 == 0 or b == S
            sizes = [b - a for a, b in r]
            assert max(sizes) - min(sizes) <= 64 + S % 64


@pytest.mark.parametrize("G", [2, 3, 8])
def test_striped_encode_equals_full(oracle, G):
    rng = np.random.default_rng(G)
    S = 64 * 37 + 38  # ragged: stripes of unequal chunk counts + a tail
    data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(30)]
    full = oracle.encode(data, 3)
    parts = [[] for _ in range(3)]
    for a, b in parallel.stripe_ranges(S, G):
        rec = oracle.encode([d[a:b] for d in data], 3)
        for j in range(3):
            parts[j].append(rec[j])
    for j in range(3):
        assert np.array_equal(np.concatenate(parts[j]), full[j])


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    elapsed = 1.0 + rank  # rank 1 is the slow one
    m = parallel.max_over_ranks(elapsed, dist)
    v = parallel.throughput(2 * 2**30, world, 10, m, "weak")
    dist.barrier()
    q.put((rank, m, v))
    dist.destroy_process_group()


def test_gloo_two_ranks_max_and_weak_throughput():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, m, v in res:
        assert m == 2.0                      # max over ranks
        assert v == pytest.approx(2 * 2 * 10 / 2.0)  # 2 ranks x 2 GiB x 10 steps / 2 s


def test_bench_launcher_two_ranks_stub():
    """bench.py --gpus 2 without torchrun: the parent spawns two rank
    processes (gloo here; the codec calls are stubbed, no GPU), the line
    reports n_gpus 2 with a world size of 2 observed by the process group, and
    value is the whole-job weak-scaling rate from the max-over-ranks time."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # --stub-legs-builtin: bench.py's own stand-ins run the legs, so rank 0's
    # c4_one_process leg runs too (c4_strong and its
    # pcie_inclusive_one_process print under the supervisor split at N > 1:
    # launcher -> one supervisor per rank -> one measurement child per rank)
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--stub-legs-builtin",
           "--segments", "8", "--segment-bytes", "65536", "--steps", "3", "--warmup", "1",
           "--settle-ms", "5", "--c4-segments", "40"]
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["world_size_observed"] == 2
    assert line["scaling"] == "weak" and line["data"].startswith("STUB")
    # value = 2 ranks x (encode + decode) x 8 segments x 64 KiB x steps / max time
    want = 2 * 2 * 8 * 65536 * 3 / 2**30 / (line["ms_per_step"] * 3 / 1e3)
    assert line["value"] == pytest.approx(want, rel=0.02, abs=0.01)
    c4 = line["c4_strong"]
    assert c4["scaling"] == "strong" and c4["stripe_bytes_per_gpu"] == 32768
    assert c4["blocks"] == [30, 10]
    assert c4["pcie_inclusive_one_process"] == {"match": True, "contexts": 2, "stub": True}
    pc = line["parity_check"]
    assert pc["all_ok"] and "c4_one_process" in pc["expected"] and "aborted" not in pc


def test_bench_refuses_mismatched_world(monkeypatch):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--stub"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=root)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def test_launcher_fails_fast_when_a_rank_dies():
    """rank 1 exits 3 right after joining the process
    group; the launcher must notice, terminate rank 0 (which would otherwise
    sit in a barrier until the process-group timeout) and return 3 within
    seconds, naming the rank."""
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--stub",
           "--segments", "8", "--segment-bytes", "65536", "--steps", "3", "--warmup", "1",
           "--settle-ms", "5", "--c4", "off"]
    env = dict(os.environ, BENCH_FAIL_RANK="1")
    env.pop("WORLD_SIZE", None)
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=150, env=env, cwd=root)
    took = time.time() - t0
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "rank 1 exited 3" in r.stderr
    assert took < 90, took  # imports dominate; the process-group timeout is 180 s
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_stub_line_reports_rank_devices_and_host_budget():
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--stub",
           "--segments", "8", "--segment-bytes", "65536", "--steps", "2", "--warmup", "1",
           "--settle-ms", "5", "--c4-segments", "40"]
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert [d["rank"] for d in line["rank_devices"]] == [0, 1]
    hb = line["host_budget"]
    assert hb["ranks"] == 2 and hb["pinned_bytes_per_rank"] == 0  # the stub pins nothing
    assert hb["pinned_bytes_node"] == 0


def test_host_budget_at_eight_ranks():
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    hb = bench.host_budget(bench.parse(["--gpus", "8"]), 8)
    # c4_strong.pcie_inclusive pins each rank's 4 MiB stripes of config 4's
    # 320 data + 33 parity + 33 restored shards
    assert hb["c4_pcie_pinned_bytes_per_rank"] == (320 + 66) * 4 * 2**20
    assert hb["rank0_c4_one_process_bytes"] == (320 + 66) * 32 * 2**20
    assert hb["pinned_bytes_node"] == 8 * hb["pinned_bytes_per_rank"] + hb["rank0_c4_one_process_bytes"]
    assert hb["mem_total"] and hb["fits"] in (True, False)


def test_torchrun_rank_failure_ends_the_job():
    """The driver's N>1 launch (torch.distributed.run): a rank that dies after
    joining the process group ends the job within seconds with a non-zero
    exit, well inside the process-group timeout (bench.PG_TIMEOUT_S)."""
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(root, "bench.py"), "--gpus", "4", "--stub", "--segments", "8",
           "--segment-bytes", "65536", "--steps", "3", "--warmup", "1", "--settle-ms", "5",
           "--c4-segments", "40"]
    env = dict(os.environ, BENCH_FAIL_RANK="2")
    env.pop("WORLD_SIZE", None)
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=170, env=env, cwd=root)
    assert r.returncode != 0
    assert time.time() - t0 < 120
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_torchrun_two_ranks_supervised_line():
    """The driver's N>1 launch form (torch.distributed.run, world 2, gloo,
    stubbed codec and legs): every rank process is a GPU-free supervisor of
    its own measurement child (round 5); exactly one line reaches stdout,
    with both ranks observed, c4_strong and its one-process figure."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(root, "bench.py"), "--gpus", "2", "--stub-legs-builtin", "--segments", "8",
           "--segment-bytes", "65536", "--steps", "3", "--warmup", "1", "--settle-ms", "5",
           "--c4-segments", "40"]
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["world_size_observed"] == 2
    assert line["parity_check"]["all_ok"] and len(line["rank_ms_per_step"]) == 2
    assert line["c4_strong"]["pcie_inclusive_one_process"]["match"] is True
    # the N>1 line carries c4_strong's own check and one
    # device per rank (distinct ordinals: cuda:LOCAL_RANK on a real node)
    assert line["c4_strong"]["parity_check"]["decode"]["match"] is True
    assert "c4_one_process" in line["parity_check"]["expected"]
    devs = line["rank_devices"]
    assert sorted(d["rank"] for d in devs) == [0, 1]
    assert len({d["stub_ordinal"] for d in devs}) == 2

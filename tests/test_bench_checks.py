"""CPU: bench.py's post-timing correctness checks (the `parity_check` object
of every bench line) flag a wrong byte, on CPU tensors standing in for the
device buffers."""
import hashlib
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _rows(n, S, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (n, S), dtype=torch.uint8, generator=g)


def test_parity_golden_check_matches_and_flags(monkeypatch):
    shapes, S, seed = [3, 2], 256, 7
    rows = _rows(3 * len(shapes), S, 1)
    golden = {"blocks": shapes, "segment_size": S, "seed": seed,
              "parity_sha256": [[hashlib.sha256(rows[3 * b + j].numpy().tobytes()).hexdigest()
                                 for j in range(3)] for b in range(len(shapes))]}
    monkeypatch.setattr(bench, "golden_parity", lambda name: golden)
    ok = bench.check_parity_golden(rows, shapes, S, seed, "x")
    assert ok["match"] and ok["shards"] == 6 and ok["mismatched"] == []
    bad = rows.clone()
    bad[4, 17] ^= 1
    r = bench.check_parity_golden(bad, shapes, S, seed, "x")
    assert not r["match"] and r["mismatched"] == [[1, 1]]
    # a batch the golden does not cover is not checked (None), never "ok"
    assert bench.check_parity_golden(rows, shapes, S, seed + 1, "x") is None
    assert bench.check_parity_golden(rows, [5], S, seed, "x") is None


def test_golden_entries_exist_for_the_bench_configs():
    from bfrs import synth
    c2 = bench.golden_parity("c2_128x32MiB")
    c4 = bench.golden_parity("c4_320x32MiB")
    assert c2["blocks"] == synth.block_shapes(128) and c2["seed"] == 0xB10C
    assert c4["blocks"] == synth.block_shapes(320) and c4["seed"] == 0xB10C
    assert c2["segment_size"] == c4["segment_size"] == 32 * 1024 * 1024


class _Sets:
    torch_equal = staticmethod(torch.equal)

    def __init__(self):
        self.shapes = [4, 3]
        self.erased = [[0, 2], [1]]
        self.data = _rows(7, 64, 3)
        self.restored = torch.zeros(6, 64, dtype=torch.uint8)
        self.restored[0] = self.data[0]
        self.restored[1] = self.data[2]
        self.restored[3] = self.data[4 + 1]


def test_restored_check_flags_a_wrong_shard():
    s = _Sets()
    r = bench.check_restored(s)
    assert r["match"] and r["restored_shards"] == 3
    s.restored[1, 5] ^= 0x80
    r = bench.check_restored(s)
    assert not r["match"] and r["mismatched"] == [[0, 2]]


@pytest.mark.parametrize("argv", [["--stub"], ["--stub", "--strong"]])
def test_stub_bench_line_carries_parity_check(argv, capfd):
    """The CPU rehearsal of the launcher prints a line with parity_check (the
    codec is a stand-in there, so the golden encode check is skipped)."""
    import json
    import subprocess
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv, "--segments", "4",
                        "--segment-bytes", "4096", "--steps", "2", "--warmup", "1",
                        "--settle-ms", "0", "--c4", "off"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    pc = line["parity_check"]
    assert pc["c3_decode"]["match"] and pc["all_ok"] and pc["ranks_ok"] == [True]
    assert pc["c2_encode"] is None


def test_live_pmc_passes_parse_and_correct(monkeypatch):
    """roofline.traffic measured in the run: bench.py runs two rocprofv3 --pmc
    child passes; stand in for rocprofv3 with a CSV of the shape it writes and
    check the dispatch filter (full-size gf_apply only) and the corrections
    (KiB, gfx950 FETCH_SIZE x2)."""
    import csv
    import shutil
    import subprocess as sp
    calls = []

    def fake_call(cmd, stdout=None, stderr=None, env=None, cwd=None):
        calls.append(cmd)
        assert cmd[:4] == ["timeout", "-s", "KILL", str(bench.PMC_PASS_TIMEOUT_S)]
        assert "--traffic-probe" in cmd and cmd[cmd.index("--") + 1] == sys.executable
        # the probe is bench.py itself (round 6: the legs moved to bench_legs.py)
        assert os.path.basename(cmd[cmd.index("--") + 2]) == "bench.py"
        assert "TORCHELASTIC_RUN_ID" not in env and env["WORLD_SIZE"] == "1"
        counter = cmd[cmd.index("--pmc") + 1]
        out = os.path.join(cmd[cmd.index("-d") + 1], "host", "123")
        os.makedirs(out)
        rows = [("fill_kernel", 4096, 1, 5.0),
                ("void bfrs::gf_apply_unrolled_kernel<true, 6, 4>(bfrs::KernArgs)", 5242880, 2, 1000.0),
                ("void bfrs::gf_apply_unrolled_kernel<true, 6, 4>(bfrs::KernArgs)", 5242880, 3, 1002.0),
                ("void bfrs::gf_apply_unrolled_kernel<true, 6, 4>(bfrs::KernArgs)", 5242880, 4, 998.0),
                ("void bfrs::gf_tail_kernel(bfrs::KernArgs)", 256, 5, 1.0)]
        with open(os.path.join(out, "pmc_counter_collection.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Dispatch_Id", "Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value"])
            for name, grid, d, v in rows:
                # two dimension rows per dispatch, summed by the parser
                w.writerow([d, name, grid, counter, v / 2])
                w.writerow([d, name, grid, counter, v / 2])
        return 0

    monkeypatch.setattr(sp, "call", fake_call)
    monkeypatch.setattr(shutil, "which", lambda name: "/usr/bin/" + name)
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "x")
    args = bench.parse(["--segments", "128"])
    traffic, src = bench.live_pmc_traffic(args)
    assert [c[c.index("--pmc") + 1] for c in calls] == ["FETCH_SIZE", "WRITE_SIZE"]
    assert src["dispatches"] == [3, 3]
    assert src["hbm_read_bytes_per_launch"] == 1000 * 1024 * 2
    assert src["hbm_write_bytes_per_launch"] == 1000 * 1024
    assert traffic == 3000 * 1024

    def failing(cmd, **kw):
        return 137
    monkeypatch.setattr(sp, "call", failing)
    traffic, src = bench.live_pmc_traffic(args)
    assert traffic is None and "exited 137" in src["error"]


def test_live_pmc_skipped_under_rocprof(monkeypatch):
    monkeypatch.setenv("ROCPROF_OUTPUT_PATH", "/tmp/x")
    assert bench.under_rocprof()
    monkeypatch.delenv("ROCPROF_OUTPUT_PATH")
    for k in [k for k in os.environ if k.startswith("ROCPROF_")]:
        monkeypatch.delenv(k)
    assert not bench.under_rocprof()


def test_rayon_fresh_process_child(monkeypatch):
    """crate_api.generate_parity_all_blocks_fresh_process: the child's JSON line
    is mapped to the bench's fields, and a failing child becomes an error
    entry, never an exception."""
    import json
    import subprocess as sp

    class R:
        def __init__(self, rc, out, err=""):
            self.returncode, self.stdout, self.stderr = rc, out, err
    line = {"link_floor_ms": 84.5, "seen_pinned": [90.0, 91.0], "fresh_pinned": [92.0, 95.0],
            "fresh_pinned_GiBps": 43.5, "seen_pinned_GiBps": 44.4}
    seen = {}

    def ok_run(cmd, capture_output, text, env, cwd):
        seen["cmd"], seen["env"] = cmd, env
        return R(0, "progress\n" + json.dumps(line) + "\n")
    monkeypatch.setattr(sp, "run", ok_run)
    r = bench.rayon_fresh_process()
    assert seen["cmd"][:4] == ["timeout", "-s", "KILL", "90"]
    assert seen["cmd"][-1].endswith(os.path.join("tools", "rayon_probe.py"))
    assert seen["env"]["PROBE_MODES"] == "pinned"
    assert (r["ms"], r["median_ms"], r["inputs_seen_before_ms"], r["link_floor_ms"]) == (92.0, 95.0, 90.0, 84.5)
    monkeypatch.setattr(sp, "run", lambda *a, **k: R(137, "", "killed"))
    assert "exited 137" in bench.rayon_fresh_process()["error"]
    monkeypatch.setattr(sp, "run", lambda *a, **k: R(0, "not json"))
    assert "error" in bench.rayon_fresh_process()


def test_c4_stripes_reassembled_for_the_golden_check(monkeypatch):
    """N > 1: c4_strong's parity stripes are all-gathered after the timed
    region and rank 0 checks the reassembled whole shards against the golden
    digests; a wrong byte in another rank's stripe is caught."""
    from bfrs import parallel
    shapes, S, world = [3, 2], 384, 3
    whole = _rows(3 * len(shapes), S, 5)
    golden = {"blocks": shapes, "segment_size": S, "seed": 0xB10C,
              "parity_sha256": [[hashlib.sha256(whole[3 * b + j].numpy().tobytes()).hexdigest()
                                 for j in range(3)] for b in range(len(shapes))]}
    monkeypatch.setattr(bench, "golden_parity", lambda name: golden)
    ranges = parallel.stripe_ranges(S, world)
    assert len({hi - lo for lo, hi in ranges}) >= 1 and ranges[-1][1] == S

    def fake_rt(stripes):
        class Dist:
            @staticmethod
            def all_gather(parts, mine):
                for g, p in enumerate(parts):
                    p.zero_()
                    p[:, :stripes[g].shape[1]].copy_(stripes[g])

        class RT:
            rank, coll_device = 0, "cpu"
            dist = Dist()
        rt = RT()
        rt.world, rt.torch = world, torch
        return rt

    stripes = [whole[:, lo:hi].clone() for lo, hi in ranges]
    r = bench.check_c4_stripes_golden(fake_rt(stripes), stripes[0], shapes, S)
    assert r["match"] and r["assembled_from_ranks"] == world and r["shards"] == 6
    stripes[2][4, 3] ^= 0x10  # block 1, parity 1, in the last rank's stripe
    r = bench.check_c4_stripes_golden(fake_rt(stripes), stripes[0], shapes, S)
    assert not r["match"] and r["mismatched"] == [[1, 1]]


# ---------------------------------------------------------------- all_ok
def _stub_legs(monkeypatch, **override):
    """Stand-ins for the N=1 legs, each reporting a passing check; `override`
    replaces some of them."""
    legs = {
        "check_config1": lambda ctx: {"match": True},
        "blake3_device": lambda ctx, sets: {"GBps": 1.0, "parity_check": {"match": True}},
        "pcie_inclusive": lambda ctx, sets: {"decode_match": True},
        "crate_api": lambda ctx, sets: {"recover_match": True},
        "cpu_baseline": lambda args, sets, info: {"self_check": True, "value": 1.0},
        "run_c5": lambda args, ctx: {"blake3_match": True, "repair": {"match": True}},
        "c4_one_process": lambda args, ctx, world, one: {"match": True},
    }
    legs.update(override)
    for k, v in legs.items():
        monkeypatch.setattr(bench, k, v)


def _run_stub_main(capsys):
    import json
    rc = bench.main(["--stub", "--stub-legs", "--segments", "4", "--segment-bytes", "4096",
                     "--steps", "2", "--warmup", "1", "--settle-ms", "0", "--c4-segments", "40"])
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    return rc, line


def test_all_legs_passing_gives_all_ok(monkeypatch, capsys):
    _stub_legs(monkeypatch)
    rc, line = _run_stub_main(capsys)
    pc = line["parity_check"]
    assert rc == 0 and pc["all_ok"] and pc["failed"] == []
    for k in ("c1_rs13", "c3_decode", "c5_blake3", "c5_repair", "blake3_c2", "pcie_decode",
              "crate_recover", "cpu_baseline_self_check", "c4_decode", "c4_one_process"):
        assert k in pc["expected"], k
    assert "c2_encode" in pc["not_applicable"]  # no golden covers a 4 x 4 KiB batch


def test_c5_error_entry_fails_the_line(monkeypatch, capsys):
    _stub_legs(monkeypatch, run_c5=lambda args, ctx: {"error": "OSError: [Errno 28] No space"})
    rc, line = _run_stub_main(capsys)
    pc = line["parity_check"]
    assert rc != 0 and not pc["all_ok"]
    assert set(pc["failed"]) == {"c5_blake3", "c5_repair"}


def test_blake3_bfrs_error_fails_the_line_and_skips_later_legs(monkeypatch, capsys):
    import bfrs
    ran = []

    def b3(ctx, sets):
        raise bfrs.BfrsError(-11, "hip: an illegal memory access was encountered")

    def crate(ctx, sets):
        ran.append("crate")
        return {"recover_match": True}
    _stub_legs(monkeypatch, blake3_device=b3, crate_api=crate)
    rc, line = _run_stub_main(capsys)
    pc = line["parity_check"]
    assert rc != 0 and not pc["all_ok"]
    assert "blake3_c2" in pc["failed"] and "blake3_device_ran" in pc["failed"]
    assert "BfrsError" in line["blake3_device"]["error"]
    assert pc["aborted"].startswith("blake3_device raised BfrsError")
    assert ran == [] and "skipped" in line["crate_api"]["error"]


def test_a_check_that_did_not_run_fails(monkeypatch, capsys):
    # a leg that returns without its check value (None) must not pass
    _stub_legs(monkeypatch, pcie_inclusive=lambda ctx, sets: {"encode_GiBps": 50.0})
    rc, line = _run_stub_main(capsys)
    assert rc != 0 and line["parity_check"]["failed"] == ["pcie_decode"]


def test_parity_summary_rules():
    s = bench.parity_summary({"a": (True, True), "b": (True, None), "c": (False, None),
                              "d": (True, False)}, {})
    assert s["failed"] == ["b", "d"] and s["not_applicable"] == ["c"] and not s["all_ok"]
    assert bench.leg_flag({"error": "x"}, "match") is False
    assert bench.leg_flag(None, "match") is False
    assert bench.leg_flag({"r": {"match": True}}, "r", "match") is True


# ---------------------------------------------------------------- roofline.trace
def _write_trace(path, launches, grid=5242880):
    import csv
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kind", "Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp",
                    "Grid_Size_X"])
        t = 1000
        w.writerow(["KERNEL_DISPATCH", 0, "fill_kernel", t, t + 50, 4096])
        for i, dur_ns in enumerate(launches):
            t += 10_000
            w.writerow(["KERNEL_DISPATCH", i + 1,
                        "void bfrs::gf_apply_unrolled_kernel<true, 6, 4>(bfrs::KernArgs)",
                        t, t + dur_ns, grid])
            t += dur_ns
        w.writerow(["KERNEL_DISPATCH", 999,
                    "void bfrs::gf_apply_unrolled_kernel<true, 6, 4>(bfrs::KernArgs)", t, t + 7, 256])


def test_kernel_trace_summary_takes_the_timed_region(tmp_path):
    p = str(tmp_path / "run_kernel_trace.csv")
    # 6 settle/warmup launches at 1.2 ms, then 2K = 4 timed launches at 0.8 ms
    _write_trace(p, [1_200_000] * 6 + [800_000, 800_000, 790_000, 810_000])
    s = bench.summarize_kernel_trace(p, steps=2)
    assert s["launches"] == 4 and s["launches_in_trace"] == 10
    assert s["mean_ms"] == 0.8 and s["median_ms"] == 0.8 and s["grid"] == 5242880
    assert "gf_apply_unrolled_kernel" in s["kernel"]
    with pytest.raises(RuntimeError):
        bench.summarize_kernel_trace(p, steps=6)


def test_live_kernel_trace_child_pass(monkeypatch, tmp_path):
    import shutil
    import subprocess as sp
    seen = {}

    def fake_call(cmd, stdout=None, stderr=None, env=None, cwd=None):
        seen["cmd"] = cmd
        assert cmd[:4] == ["timeout", "-s", "KILL", str(bench.TRACE_PASS_TIMEOUT_S)]
        i = cmd.index("--")
        assert cmd[i + 1] == sys.executable and "--trace-probe" in cmd  # no shell hop
        assert os.path.basename(cmd[i + 2]) == "bench.py"
        assert "--kernel-trace" in cmd[:i] and "--stats" in cmd[:i] and "--pmc" not in cmd
        out = os.path.join(cmd[cmd.index("-d") + 1], "host", "1")
        os.makedirs(out)
        _write_trace(os.path.join(out, "run_kernel_trace.csv"), [900_000] * 4 + [820_000] * 6)
        with open(os.path.join(out, "run_kernel_stats.csv"), "w") as f:
            f.write('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"\n'
                    '"void bfrs::gf_apply_unrolled_kernel<true, 6, 4>(bfrs::KernArgs)",10,8,820000.0,90.0,1,2,3\n')
        stdout.write('{"launch_ms": 0.8213, "steps": 3, "ms_per_step": 1.7}\n')
        return 0
    monkeypatch.setattr(sp, "call", fake_call)
    monkeypatch.setattr(shutil, "which", lambda name: "/usr/bin/" + name)
    args = bench.parse(["--steps", "3", "--warmup", "2"])
    prof = str(tmp_path / "prof")
    s = bench.live_kernel_trace(args, prof)
    assert "error" not in s, s
    assert s["launches"] == 6 and s["mean_ms"] == 0.82 and s["child_event_launch_ms"] == 0.8213
    assert s["stats_top"][0]["average_ms"] == 0.82
    assert os.path.exists(os.path.join(prof, "trace_kernel_stats.csv"))
    assert os.path.exists(os.path.join(prof, "trace_c2_launch_summary.json"))
    monkeypatch.setattr(sp, "call", lambda cmd, **kw: 124)
    assert "exited 124" in bench.live_kernel_trace(args)["error"]


# ---------------------------------------------------------------- supervisor
def test_supervisor_keeps_the_line_when_the_child_segfaults():
    """The measurement child dies by SIGSEGV inside a leg after the timed
    region: the GPU-free parent still prints the line with the completed
    legs, names the leg and the signal in parity_check.aborted, sets all_ok
    false and exits non-zero (128 + 11); faulthandler printed the stack."""
    import json
    import subprocess
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--stub-legs-builtin",
                        "--segments", "4", "--segment-bytes", "4096", "--steps", "2",
                        "--warmup", "1", "--settle-ms", "0", "--c4", "off",
                        "--stub-crash-leg", "pcie_inclusive"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 139, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    pc = line["parity_check"]
    assert pc["aborted"] == "pcie_inclusive: SIGSEGV" and pc["all_ok"] is False
    assert "leg pcie_inclusive" in pc["failed"]
    assert line["value"] > 0 and line["ms_per_step"] > 0  # the headline survived
    assert line["blake3_device"]["stub"]                   # a leg done before the crash
    assert "died in this leg" in line["pcie_inclusive"]["error"]
    assert "crate_api" not in line                          # never started
    assert "Fatal Python error: Segmentation fault" in r.stderr
    assert "in leg" in r.stderr


def test_supervisor_passes_a_complete_line_through():
    import json
    import subprocess
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--stub-legs-builtin",
                        "--segments", "4", "--segment-bytes", "4096", "--steps", "2",
                        "--warmup", "1", "--settle-ms", "0", "--c4", "off"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    pc = line["parity_check"]
    assert pc["all_ok"] and "aborted" not in pc and pc["failed"] == []
    for key in ("blake3_device", "pcie_inclusive", "crate_api", "cpu_baseline", "c5"):
        assert line[key]["stub"], key


def test_finish_supervised_rules(capsys):
    import json
    base = {"value": 4800.0, "parity_check": {"failed": [], "all_ok": True}}
    # a final line: printed as written, with the child's own code
    assert bench.finish_supervised({"line": dict(base), "final": True}, 0) == 0
    assert json.loads(capsys.readouterr().out)["value"] == 4800.0
    # a final line, then a crash in the teardown: flagged, non-zero
    rc = bench.finish_supervised({"line": json.loads(json.dumps(base)), "final": True}, -11)
    out = json.loads(capsys.readouterr().out)
    assert rc == 139 and out["parity_check"]["aborted"] == "after the line: SIGSEGV"
    assert out["parity_check"]["all_ok"] is False
    # a checkpoint between legs, child killed
    rc = bench.finish_supervised({"line": json.loads(json.dumps(base)), "final": False,
                                  "running": None}, -9)
    out = json.loads(capsys.readouterr().out)
    assert rc == 137 and out["parity_check"]["aborted"] == "between legs: SIGKILL"
    # an exit code instead of a signal, inside a leg
    rc = bench.finish_supervised({"line": json.loads(json.dumps(base)), "final": False,
                                  "running": "c5", "running_key": "c5"}, 3)
    out = json.loads(capsys.readouterr().out)
    assert rc == 3 and out["parity_check"]["aborted"] == "c5: exit 3" and "error" in out["c5"]
    # no checkpoint at all: no line
    assert bench.finish_supervised(None, -11) == 139
    assert capsys.readouterr().out == ""


def test_supervisor_not_used_where_it_must_not_be(monkeypatch):
    for k in [k for k in os.environ if k.startswith("ROCPROF_")]:
        monkeypatch.delenv(k)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.wants_supervisor(bench.parse([]))
    assert not bench.wants_supervisor(bench.parse(["--no-supervisor"]))
    assert not bench.wants_supervisor(bench.parse(["--trace-probe"]))
    assert not bench.wants_supervisor(bench.parse(["--gpus", "2"]))  # the spawn launcher
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.wants_supervisor(bench.parse(["--gpus", "2"]))  # a rank process
    monkeypatch.setenv("ROCPROF_OUTPUT_PATH", "/tmp/x")
    assert not bench.wants_supervisor(bench.parse([]))  # the profiled process measures


def test_blake3_kernel_split_from_the_trace(tmp_path):
    import csv
    p = str(tmp_path / "t.csv")
    with open(p, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kind", "Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp",
                    "Grid_Size_X"])
        t = 0
        for call in range(3):
            w.writerow(["K", 0, "void bfrs::blake3_group_kernel<3u, 0u>(...)", t, t + 1_400_000, 1])
            w.writerow(["K", 0, "void bfrs::blake3_reduce_kernel<64u>(...)", t + 1_410_000,
                        t + 1_430_000, 1])
            w.writerow(["K", 0, "void bfrs::blake3_reduce_kernel<64u>(...)", t + 1_440_000,
                        t + 1_450_000 + call, 1])
            t += 5_000_000
    s = bench.summarize_blake3_trace(p, 3)
    assert s["group_kernel_ms"] == 1.4 and s["reduce_launches_per_call"] == 2
    assert s["reduce_kernels_ms_per_call"] == pytest.approx(0.03, abs=1e-4)
    assert s["device_span_ms"] == 1.45 and s["calls"] == 3
    assert bench.summarize_blake3_trace(p, 4) is None
    fig = bench.blake3_trace_figures({"blake3": s}, 128 * 32 * 2**20)
    assert 0 < fig["frac_group_kernel"] < 2
    assert "error" in bench.blake3_trace_figures({"error": "x"}, 1)


def test_probe_children_never_see_the_state_file(monkeypatch):
    """A probe child (PMC / trace pass, rayon probe) must neither write its
    line into the supervisor's state file nor take the measurement child's
    exit path (which skips rocprofv3's output at exit)."""
    monkeypatch.setenv(bench.STATE_ENV, "/tmp/state.json")
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "x")
    env = bench.probe_env(WORLD_SIZE="1")
    assert bench.STATE_ENV not in env and "TORCHELASTIC_RUN_ID" not in env
    assert env["WORLD_SIZE"] == "1"

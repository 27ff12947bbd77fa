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

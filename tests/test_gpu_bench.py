"""GPU: bench.py's multi-rank path end to end (the launcher, the column-stripe
partition of config C4 and the max-over-ranks reduction) with two ranks on
cuda:0 over gloo (RCCL needs one GPU per rank; the driver's 8-GPU run uses
RCCL).  The ranks' C4 parity stripes are assembled and compared with the
oracle's RS(k,3) of the full segments."""
import glob
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_strong_stripes_assemble_to_oracle_parity(oracle, tmp_path):
    from bfrs import synth
    S, nseg = 1 << 20, 40  # 1 MiB segments: blocks RS(30,3) + RS(10,3)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--one-device",
           "--backend", "gloo", "--segments", "8", "--segment-bytes", str(S), "--steps", "2",
           "--warmup", "1", "--settle-ms", "20", "--c4-segments", str(nseg),
           "--dump-dir", str(tmp_path), "--cpu-baseline", "off", "--pcie", "off",
           "--crate", "off", "--c5", "off"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["world_size_observed"] == 2
    assert line["c4_strong"]["scaling"] == "strong"
    stripes = sorted(glob.glob(str(tmp_path / "c4_stripe_rank*.json")))
    assert len(stripes) == 2
    parts = []
    for rank in range(2):
        meta = json.load(open(tmp_path / f"c4_stripe_rank{rank}.json"))
        parts.append((meta["lo"], meta["hi"], np.load(tmp_path / f"c4_parity_rank{rank}.npy")))
    shapes = synth.block_shapes(nseg)
    assert sum(hi - lo for lo, hi, _ in parts) == S
    seg = 0
    for b, k in enumerate(shapes):
        want = oracle.encode([synth.segment_np(0xB10C, seg + i, S) for i in range(k)], 3,
                             oracle.ENGINE_AVX2)
        for j in range(3):
            got = np.concatenate([p[3 * b + j] for _, _, p in parts])
            assert np.array_equal(got, want[j]), (b, j)
        seg += k


def test_driver_scale_form_at_one_rank_over_rccl():
    """The driver's SCALE command at N = 1 (`python -m torch.distributed.run
    --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 ... bench.py --gpus 1`):
    under torchrun the rank joins an RCCL process group even alone, so this
    runs the real collectives of an N > 1 line (barriers, the max-over-ranks
    all-reduce, the rank_devices all-gather) on the GPU, behind the
    supervisor, with small sizes.  One line, both C2 and C4 checks green."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "bench.py"), "--gpus", "1", "--segments", "8",
           "--segment-bytes", str(1 << 20), "--steps", "3", "--warmup", "1", "--settle-ms", "20",
           "--c4-segments", "40", "--cpu-baseline", "off", "--pcie", "off", "--crate", "off",
           "--c5", "off", "--pmc", "off", "--trace", "off"]
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["world_size_observed"] == 1
    pc = line["parity_check"]
    assert pc["all_ok"], pc
    assert line["c4_strong"]["parity_check"]["decode"]["match"] is True
    assert line["rank_devices"][0]["device"] == 0

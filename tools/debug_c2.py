"""Diagnose the C2 batch: per-block parity vs golden digests across call patterns."""
import hashlib, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blockframe-rs_amd"))
import torch, bfrs
from bfrs import synth
g = json.load(open(os.path.join(ROOT, "tests/golden/rs_large.json")))["c2_128x32MiB"]
S = g["segment_size"]; shapes = g["blocks"]; nb = len(shapes)
data = torch.empty(128, S, dtype=torch.uint8, device="cuda")
for s in range(128):
    synth.fill_segment_torch(data[s], g["seed"], s)
torch.cuda.synchronize()
ctx = bfrs.Context(0)
rec = torch.empty(3 * nb, S, dtype=torch.uint8, device="cuda")
def check(tag):
    torch.cuda.synchronize()
    ok = []
    for b in range(nb):
        ok.append(all(hashlib.sha256(rec[3*b+j].cpu().numpy().tobytes()).hexdigest() == g["parity_sha256"][b][j] for j in range(3)))
    print(tag, ok, flush=True)
def batch():
    rec.zero_()
    ctx.encode_batch_dev(shapes, 3, S, [data[s] for s in range(128)], [rec[i] for i in range(3*nb)])
batch(); check("batch#1")
batch(); check("batch#2")
rec.zero_(); seg = 0
for b, k in enumerate(shapes):
    ctx.encode_batch_dev([k], 3, S, [data[seg+i] for i in range(k)], [rec[3*b+j] for j in range(3)]); seg += k
check("single-block calls")
for t in ("1", "2", "5", "8"):
    os.environ["BFRS_TILES_PER_WG"] = t
    batch(); check(f"batch tpw={t}")
os.environ.pop("BFRS_TILES_PER_WG")
os.environ["BFRS_DEBUG_DESC"] = "1"
for i in range(10):
    batch(); check(f"batch debug-desc #{i}")

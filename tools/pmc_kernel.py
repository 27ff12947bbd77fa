"""Launch loop of ONE gf_apply variant on the bench shape, for rocprofv3 PMC
passes (measurement tool).  usage: BFRS_KERNEL_VARIANT=73 python tools/pmc_kernel.py [--decode] [--n 20]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blockframe-rs_amd"))
# the A/B variants live only in the measurement build (make -C blockframe-rs_amd/csrc ab)
os.environ.setdefault("BFRS_LIB", "libbfrs_ab.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--decode", action="store_true")
    ap.add_argument("--n", type=int, default=20)
    ap.add_argument("--segments", type=int, default=128)
    a = ap.parse_args()
    import torch
    import bfrs
    from bfrs import synth
    S = synth.SEGMENT_SIZE
    shapes = synth.block_shapes(a.segments)
    nb = len(shapes)
    data = bfrs.empty_shards(a.segments, S)
    for s in range(a.segments):
        synth.fill_segment_torch(data[s], 0xB10C, s)
    par = bfrs.empty_shards(3 * nb, S)
    rest = bfrs.empty_shards(3 * nb, S)
    dec_in, dec_out, seg = [], [], 0
    for b, k in enumerate(shapes):
        er = [1, k // 2, k - 1]
        for i in range(k):
            dec_in.append(None if i in er else data[seg + i])
            dec_out.append(rest[3 * b + er.index(i)] if i in er else None)
        seg += k
    ctx = bfrs.Context(0)
    sh = torch.cuda.current_stream().cuda_stream
    enc = ctx.prepare_encode(shapes, 3, S, [data[s] for s in range(a.segments)],
                             [par[i] for i in range(3 * nb)])
    dec = ctx.prepare_decode(shapes, 3, S, dec_in, [par[i] for i in range(3 * nb)], dec_out)
    enc(sh)
    fn = dec if a.decode else enc
    for _ in range(a.n):
        fn(sh)
    torch.cuda.synchronize()
    print("ok", os.environ.get("BFRS_KERNEL_VARIANT"), "decode" if a.decode else "encode", a.n)


if __name__ == "__main__":
    main()

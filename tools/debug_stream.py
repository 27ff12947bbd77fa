"""Which tiles does a kernel variant get wrong?  Encodes / decodes on the GPU
with the variant under test and with the default, and prints the mismatching
8 KiB tiles per output.  usage: BFRS_KERNEL_VARIANT=24 python tools/debug_stream.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blockframe-rs_amd"))


def main():
    import torch
    import bfrs
    var = os.environ.get("BFRS_KERNEL_VARIANT", "5")
    ctx = bfrs.Context(0)
    gen = torch.Generator(device="cuda").manual_seed(1)
    for (ks, n) in (([4], 8 << 20), ([1], 8 << 20), ([30], 8 << 20), ([30, 8], 4 << 20), ([30, 30, 30, 30, 8], 32 << 20)):
        data = [torch.randint(0, 256, (k, n), dtype=torch.uint8, device="cuda", generator=gen) for k in ks]
        outs = {}
        for v in ("5", var):
            os.environ["BFRS_KERNEL_VARIANT"] = v
            par = torch.zeros(3 * len(ks), n, dtype=torch.uint8, device="cuda")
            ctx.encode_batch_dev(ks, 3, n, [d[i] for d in data for i in range(d.shape[0])],
                                 [par[j] for j in range(3 * len(ks))])
            torch.cuda.synchronize()
            outs[v] = par
        ref, got = outs["5"], outs[var]
        bad = (ref != got).view(3 * len(ks), n // 8192, 8192).any(dim=2)
        for o in range(3 * len(ks)):
            tiles = bad[o].nonzero().flatten().tolist()
            if tiles:
                print(f"ks={ks} n={n} out {o}: {len(tiles)} bad tiles, first {tiles[:12]}")
        print(f"ks={ks} n={n}: encode {'OK' if not bad.any() else 'MISMATCH'}", flush=True)
        # decode: ne erasures per block (n_out = ne), all parity present
        for ne in (1, 3):
            d_orig, d_out, want = [], [], []
            for b, k in enumerate(ks):
                er = list(range(1, 1 + ne))
                for i in range(k):
                    d_orig.append(None if i in er else data[b][i])
                    if i in er:
                        t = torch.zeros(n, dtype=torch.uint8, device="cuda")
                        d_out.append(t)
                        want.append((t, data[b][i]))
                    else:
                        d_out.append(None)
            ctx.decode_batch_dev(ks, 3, n, d_orig, [ref[j] for j in range(3 * len(ks))], d_out)
            torch.cuda.synchronize()
            for wi, (t, d) in enumerate(want):
                bt = (t != d).view(n // 8192, 8192).any(dim=1).nonzero().flatten().tolist()
                if bt:
                    print(f"  decode ne={ne} restored {wi}: {len(bt)} bad tiles, first {bt[:12]}")
            print(f"ks={ks} n={n}: decode ne={ne} done", flush=True)


if __name__ == "__main__":
    main()

"""A/B timing of gf_apply variants in ONE process (interleaved rounds).

usage: python tools/kbench.py [--rounds R] [--iters N] [--variants 41,5,44] [--tpw 1,2,5]
A variant "V:io" runs kernel V in io mode enc / dec / encdr (an encode over the
decode's regions: survivors + parity rows in, restored rows out) / encr (data in,
restored rows out): memory-region diagnosis, outputs not checked.
Variant 44 is a traffic-only probe (no GF arithmetic, wrong output): it gives the
ceiling of this exact access pattern.  Also times a torch device copy.
"""
import argparse
import json
import os
import sys
import time

PROBES = ("44", "72", "74")  # traffic-only probes: no codec output to check
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blockframe-rs_amd"))
# the A/B variants live only in the measurement build (make -C blockframe-rs_amd/csrc ab)
os.environ.setdefault("BFRS_LIB", "libbfrs_ab.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--variants", default="41,5,44")
    ap.add_argument("--tpw", default="0")
    ap.add_argument("--segments", type=int, default=128)
    ap.add_argument("--decode", action="store_true")
    ap.add_argument("--copy-probe", action="store_true",
                    help="also time a torch copy inside each layout's first buffer (placement study)")
    ap.add_argument("--settle-ms", type=float, default=200.0,
                    help="untimed launches of the same config right before each timed run")
    ap.add_argument("--stagger", default="0",
                    help="comma list: extra bytes between consecutive shards (row pitch S + x); "
                         "suffix b = block-interleaved rows (each block's k data, 3 parity and "
                         "3 restored rows consecutive in one buffer, as the archive arenas); "
                         "suffix c = physically contiguous allocations (hipDeviceMallocContiguous); "
                         "suffix s = data, parity and restored rows in one allocation; suffix r = every row its own allocation")
    ap.add_argument("--pad-gib", type=float, default=0.0,
                    help="allocate (and keep) this much HBM before the layouts: does a layout's "
                         "placement mode follow its allocation order? (round 6)")
    a = ap.parse_args()
    import numpy as np
    import torch
    pad = (torch.empty(int(a.pad_gib * 2**30), dtype=torch.uint8, device="cuda")
           if a.pad_gib > 0 else None)
    import bfrs
    from bfrs import synth
    os.environ["BFRS_ALLOW_PROBE"] = "1"
    S = synth.SEGMENT_SIZE
    shapes = synth.block_shapes(a.segments)
    nb = len(shapes)
    keep = []  # contiguous allocations stay alive for the whole run

    def contiguous_buffer(nbytes):
        """hipExtMallocWithFlags(hipDeviceMallocContiguous) wrapped as a torch
        tensor: physically contiguous, so the row stagger maps onto HBM
        channels the same way on every box (layout A/B, suffix c)."""
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        ptr = ctypes.c_void_p()
        rc = hip.hipExtMallocWithFlags(ctypes.byref(ptr), ctypes.c_size_t(nbytes), ctypes.c_uint(0x4))
        if rc != 0:
            raise RuntimeError(f"hipExtMallocWithFlags(contiguous, {nbytes}) = {rc}")

        class CAI:
            __cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1",
                                        "data": (ptr.value, False), "version": 2}
        t = torch.as_tensor(CAI(), device="cuda")
        keep.append((hip, ptr))
        return t

    def rows(n, pitch, contiguous=False):
        """n shard views of S bytes, row i at byte i * pitch of one buffer."""
        buf = (contiguous_buffer(n * pitch) if contiguous
               else torch.empty(n * pitch, dtype=torch.uint8, device="cuda"))
        bufs.append(buf)
        return [buf[i * pitch:i * pitch + S] for i in range(n)]

    bufs = []  # the flat buffer behind each rows() call (copy probe)

    def build(x):
        del bufs[:]
        x = x.split("#")[0]  # "#n": another copy of the same layout (placement study)
        contig = x.endswith("c")
        x = x.rstrip("c")
        single = x.endswith("s")
        x = x.rstrip("s")
        per_row = x.endswith("r")
        x = x.rstrip("r")
        stagger = int(x.rstrip("b"))
        if per_row:  # every shard row its own allocation
            def one(n):
                out = []
                for _ in range(n):
                    b_ = torch.empty(S + stagger, dtype=torch.uint8, device="cuda")
                    bufs.append(b_)
                    out.append(b_[:S])
                return out
            data, par, rest = one(a.segments), one(3 * nb), one(3 * nb)
        elif single:  # data, parity and restored rows in ONE allocation (bench --layout single)
            allr = rows(a.segments + 6 * nb, S + stagger, contig)
            data, par, rest = allr[:a.segments], allr[a.segments:a.segments + 3 * nb], \
                allr[a.segments + 3 * nb:]
        elif x.endswith("b"):
            allr = rows(sum(k + 6 for k in shapes), S + stagger, contig)
            data, par, rest, r = [], [], [], 0
            for k in shapes:
                data += allr[r:r + k]
                par += allr[r + k:r + k + 3]
                rest += allr[r + k + 3:r + k + 6]
                r += k + 6
        else:
            data = rows(a.segments, S + stagger, contig)
            par = rows(3 * nb, S + stagger, contig)
            rest = rows(3 * nb, S + stagger, contig)
        for s_ in range(a.segments):
            synth.fill_segment_torch(data[s_], 0xB10C, s_)
        dec_in, dec_out, seg, erased = [], [], 0, []
        for b, k in enumerate(shapes):
            er = [1, k // 2, k - 1]
            for i in range(k):
                dec_in.append(None if i in er else data[seg + i])
                dec_out.append(rest[3 * b + er.index(i)] if i in er else None)
                if i in er:
                    erased.append((3 * b + er.index(i), seg + i))
            seg += k
        dr_in, seg = [], 0  # per block: surviving data rows, then its 3 parity rows
        for b, k in enumerate(shapes):
            dr_in += [x for x in dec_in[seg:seg + k] if x is not None] + par[3 * b:3 * b + 3]
            seg += k
        return dict(data=data, par=par, rest=rest, dec_in=dec_in, dec_out=dec_out, erased=erased,
                    dr_in=dr_in, flat=bufs[0])

    layouts = {x: build(x) for x in a.stagger.split(",")}
    ctx = bfrs.Context(0)
    stream = torch.cuda.current_stream()
    alg = sum(k + 3 for k in shapes) * S

    def run(L, io=None):
        io = io or ("dec" if a.decode else "enc")
        if io == "dec":
            ctx.decode_batch_dev(shapes, 3, S, L["dec_in"], L["par"], L["dec_out"], stream=stream)
        elif io == "enc":
            ctx.encode_batch_dev(shapes, 3, S, L["data"], L["par"], stream=stream)
        elif io == "encdr":  # an encode over the decode's regions: survivors + parity in, restored out
            ctx.encode_batch_dev(shapes, 3, S, L["dr_in"], L["rest"], stream=stream)
        elif io == "encr":  # an encode writing the restored rows instead of the parity rows
            ctx.encode_batch_dev(shapes, 3, S, L["data"], L["rest"], stream=stream)
        else:
            raise SystemExit(f"unknown io mode {io}")

    os.environ["BFRS_KERNEL_VARIANT"] = "76"
    os.environ.pop("BFRS_TILES_PER_WG", None)
    for L in layouts.values():
        ctx.encode_batch_dev(shapes, 3, S, L["data"], L["par"], stream=stream)  # parity for decode
        run(L)
    torch.cuda.synchronize()
    L0 = next(iter(layouts.values()))
    ref = torch.stack(L0["par"]).clone()
    t0 = time.perf_counter()  # clock settle (~1 s of launches)
    while time.perf_counter() - t0 < 1.0:
        for _ in range(16):
            run(L0)
        torch.cuda.synchronize()
    configs = [(v, t, x) for v in a.variants.split(",") for t in a.tpw.split(",") for x in layouts]
    res = {c: [] for c in configs}
    src = L0["data"][0].new_empty(alg // 2)
    dst = torch.empty_like(src)
    copy_ms = []
    import random
    rng = random.Random(0x5EED)

    def select(v, t):
        os.environ["BFRS_KERNEL_VARIANT"] = v.split(":")[0]
        if t == "0":
            os.environ.pop("BFRS_TILES_PER_WG", None)
        else:
            os.environ["BFRS_TILES_PER_WG"] = t

    for r in range(a.rounds):
        order = list(configs)
        rng.shuffle(order)
        for (v, t, x) in order:
            L = layouts[x]
            select(v, t)
            # settle: keep the GPU busy on this config right up to the timed
            # launches (an idle gap or host check puts the next ~30 launches
            # on ramping clocks)
            t1 = time.perf_counter()
            io = v.split(":")[1] if ":" in v else None
            while time.perf_counter() - t1 < a.settle_ms / 1e3:
                run(L, io)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.iters):
                run(L, io)
            e1.record(stream)
            torch.cuda.synchronize()
            res[(v, t, x)].append(e0.elapsed_time(e1) / a.iters)
        t1 = time.perf_counter()
        while time.perf_counter() - t1 < a.settle_ms / 1e3:
            dst.copy_(src)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(a.iters):
            dst.copy_(src)
        e1.record(stream)
        torch.cuda.synchronize()
        copy_ms.append(e0.elapsed_time(e1) / a.iters)
    # correctness of every codec variant, after the timing
    for (v, t, x) in configs:
        if v in PROBES or ":" in v:  # probes and io-mode runs have no codec output to check
            continue
        L = layouts[x]
        select(v, t)
        if a.decode:
            for t_ in L["rest"]:
                t_.zero_()
        run(L)
        torch.cuda.synchronize()
        if not a.decode:
            assert torch.equal(torch.stack(L["par"]), ref), f"variant {v} output differs"
        else:
            for ri, di in L["erased"]:
                assert torch.equal(L["rest"][ri], L["data"][di]), f"variant {v} decode differs"
    out = {}
    for (v, t, x), ms in res.items():
        m = float(np.median(ms))
        out[f"v{v}_tpw{t}" + (f"_stagger{x}" if x != "0" else "")] = {"ms": round(m, 4), "GBps": round(alg / m / 1e6, 1), "all_ms": [round(x, 4) for x in ms]}
    cm = float(np.median(copy_ms))
    out["torch_copy_same_bytes"] = {"ms": round(cm, 4), "GBps": round(alg / cm / 1e6, 1)}
    # placement probe: a plain torch copy inside each layout's first buffer
    # (first half -> second half), timed like the kernels
    if a.copy_probe:
        for x, L in layouts.items():
            fl = L["flat"]
            h = fl.numel() // 2
            src_, dst_ = fl[:h], fl[h:2 * h]
            for _ in range(5):
                dst_.copy_(src_)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.iters):
                dst_.copy_(src_)
            e1.record(stream)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            out[f"copy_in_layout_{x}"] = {"ms": round(ms, 4), "GBps": round(2 * h / ms / 1e6, 1)}
    # device addresses of each layout's first data / parity / restored row
    # (placement study: does speed follow the virtual address?)
    out["addresses"] = {x: {"data": hex(L["data"][0].data_ptr()), "par": hex(L["par"][0].data_ptr()),
                            "rest": hex(L["rest"][0].data_ptr())} for x, L in layouts.items()}
    out["pad_gib"] = a.pad_gib
    del pad
    print(json.dumps({"decode": a.decode, "alg_bytes": alg, **out}, indent=1))


if __name__ == "__main__":
    main()

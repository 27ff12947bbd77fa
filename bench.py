"""bench.py — BASELINE metric: device-resident RS(30,3) encode & 3-erasure
decode of 32 MiB segments (BASELINE.json configs[1] + configs[2]).

One step = one pass of the hot path over one batch resident in HBM:
  encode : 128 x 32 MiB segments -> 4 x RS(30,3) + 1 x RS(8,3) parity
           (exactly the blocks src/chunker/commit.rs:359,402-416 forms for a 4 GiB file)
  decode : per block, 3 data shards erased (seed 0xDEC0DE+block), restored from
           the survivors + parity (src/filestore/recovery.rs:118-173 semantics)
Both go through the C-ABI (bfrs_encode_batch_dev / bfrs_decode_batch_dev) on
torch's current stream, one kernel launch each.

value = original-data GiB processed by all ranks (encode + decode) / max-rank time.

Multi-GPU: one process per GPU.  `--gpus N` with N > 1 either runs under
torchrun (WORLD_SIZE must equal N) or, without WORLD_SIZE, spawns the N rank
processes itself before anything touches the GPU.  Every rank owns an
independent batch (weak scaling, no collective on the data path; the only
collectives are the barriers and the max-time reduction).

Sub-objects of the same JSON line:
  c4_strong    BASELINE configs[3]: 320 x 32 MiB (10 x RS(30,3) + 1 x RS(20,3)),
               64-B column stripes of every shard over the ranks (strong scaling)
  roofline     gf_apply launch time from HIP events on the launch stream;
               traffic = HBM bytes per launch from two rocprofv3 --pmc child
               passes run before the GPU is touched (N=1; the committed
               profiles/pmc_traffic.json record otherwise, named)
  cpu_baseline the oracle's AVX2 engine (restatement of reed-solomon-simd, not
               the crate) on C2's exact blocks; host CPU model and core counts
  crate_api    the crate-shaped host-memory path BlockFrame calls per block
               (bfrs_generate_parity / bfrs_recover_segment_rs30_3), and
               rayon's all-blocks shape, also in a fresh child process
  pcie_inclusive  the same batch from pinned host memory (H2D + kernel + D2H)
  c5           BASELINE configs[4]: read of a corrupted 4 GiB tier-3 archive
               through the mount's read core (bfrs_archive_read)

Process layout (round 5): run as a script, bench.py is a
GPU-free supervisor that starts the measurement as a child process (no
re-exec) and prints the line.  The child writes the line-so-far to the
supervisor's state file after the timed region and before and after every
leg, so a signal anywhere after the timed region still yields the headline,
with `parity_check.aborted` naming the leg and the signal, all_ok false and a
non-zero exit.  faulthandler is on in both processes.
"""
import argparse
import faulthandler
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "blockframe-rs_amd"))
from bench_legs import (  # noqa: E402  the side legs (bench_legs.py)
    HBM_PEAK_GBPS, PMC_FILE, STATE_ENV, probe_env,
    host_budget, check_config1, host_info, cpu_baseline,
    pcie_link, crate_api, reference_copies, B3_GOLDEN,
    B3_VALU_PER_BLOCK, B3_VALU_PER_64B_ALG, B3_LANE_OPS_PER_S, b3_ceiling_gbps,
    blake3_device, host_pressure, pinned_host_state, rayon_fresh_process,
    pcie_inclusive, PMC_PASS_TIMEOUT_S, under_rocprof, _pmc_pass,
    live_pmc_traffic, TRACE_PASS_TIMEOUT_S, B3_PROBE_CALLS, blake3_trace_figures,
    summarize_kernel_trace, summarize_blake3_trace, live_kernel_trace, pmc_traffic,
    c5_make_file, run_c5, c5_repair, c5_cpu_baseline,
    stub_leg_standins)

METRIC = "GiB/s device-resident RS(30,3) encode & 3-erasure decode, 32MB segments"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--settle-ms", type=float, default=1000.0,
                    help="untimed steps until this much wall time has passed, before the W "
                         "warmup steps: the GPU's clocks ramp over the first ~30 launches "
                         "(rocprof trace: 1.33 ms -> 0.92 ms per launch)")
    ap.add_argument("--segments", type=int, default=128, help="segments per GPU (C2: 128)")
    ap.add_argument("--segment-bytes", type=int, default=32 * 1024 * 1024)
    ap.add_argument("--pitch", type=int, default=-1,
                    help="shard row pitch in bytes (-1 = bfrs_shard_pitch; A/B of the HBM layout)")
    ap.add_argument("--layout", choices=["single", "separate"], default="separate",
                    help="shard sets in one device allocation or one each")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads for the all-cores CPU variants (0 = this host's CPU share)")
    ap.add_argument("--pcie", choices=["auto", "off"], default="auto",
                    help="also time the host-memory path (pinned buffers, H2D+kernel+D2H)")
    ap.add_argument("--crate", choices=["auto", "off"], default="auto",
                    help="time the crate-shaped per-block host API (N=1)")
    ap.add_argument("--c4", choices=["auto", "off"], default="auto",
                    help="c4_strong sub-object (configs[3], strong scaling over the ranks)")
    ap.add_argument("--c4-segments", type=int, default=320)
    ap.add_argument("--c5", choices=["auto", "off"], default="auto",
                    help="c5 sub-object (configs[4], N=1)")
    ap.add_argument("--strong", action="store_true",
                    help="value = config C4 (default 320 segments) column-striped over the ranks")
    ap.add_argument("--workload", choices=["c2c3", "c5"], default="c2c3",
                    help="c5 = only the BASELINE configs[4] read-path line")
    ap.add_argument("--c5-gib", type=float, default=4.0, help="c5 file size (SURVEY C5: 4 GiB)")
    ap.add_argument("--c5-read-bytes", type=int, default=128 << 10, help="FUSE max_read")
    ap.add_argument("--c5-dir", default=None, help="scratch directory (default $TMPDIR)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="process-group backend (nccl = RCCL on ROCm)")
    ap.add_argument("--one-device", action="store_true",
                    help="every rank uses device 0 (tests: 2 ranks on one GPU over gloo)")
    ap.add_argument("--dump-dir", default=None,
                    help="each rank writes its C4 parity stripes here (tests assemble them)")
    ap.add_argument("--pmc", choices=["auto", "off"], default="auto",
                    help="N=1: measure roofline.traffic live with two rocprofv3 --pmc child "
                         "passes before the timed run (off: the committed profiles/ record)")
    ap.add_argument("--trace", choices=["auto", "off"], default="auto",
                    help="N=1: roofline.trace from a rocprofv3 --kernel-trace --stats child pass "
                         "over the bench's own device loop, before the timed run")
    ap.add_argument("--profile-dir", default=None,
                    help="keep the trace pass's kernel stats and C2 launch summary here")
    ap.add_argument("--traffic-probe", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--trace-probe", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--stub-legs", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--stub", action="store_true",
                    help="CPU-only rehearsal of the launcher/partition/timing path: no GPU, "
                         "the codec calls replaced by a stand-in (tests only, never a bench line)")
    ap.add_argument("--no-supervisor", action="store_true",
                    help="run the measurement in this process (no GPU-free parent)")
    ap.add_argument("--stub-crash-leg", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--stub-legs-builtin", action="store_true", help=argparse.SUPPRESS)
    a = ap.parse_args(argv)
    if a.stub_legs_builtin:  # a subprocess test: bench.py's own stand-ins run the legs
        a.stub = a.stub_legs = True
    if a.strong and a.segments == 128:
        a.segments = 320
    if a.stub:
        a.backend = "gloo"
        a.pmc = a.trace = "off"
        if not a.stub_legs:  # --stub-legs: tests stand in for the N=1 legs themselves
            a.cpu_baseline = a.pcie = a.crate = a.c5 = "off"
    return a


T_START = time.perf_counter()


# The JSON line's channel.  Run as a script, stdout carries nothing else
# (claim_stdout): C++ code in the process (gloo prints its "[Gloo] Rank ...
# connected" lines to fd 1, RCCL its debug output) writes to stderr instead.
JSON_OUT = None


def claim_stdout():
    global JSON_OUT
    sys.stdout.flush()
    JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)


def emit(obj):
    """The line: printed on the JSON channel, or, in the supervisor's
    measurement child, written as the final state for the supervisor to print."""
    if STATE.path:
        STATE.line = obj
        STATE.save(final=True)
        return
    print(json.dumps(obj), file=JSON_OUT or sys.stdout, flush=True)


def progress(msg):
    """One stderr line per bench phase (a long run shows it is alive)."""
    print(f"bench.py [{time.perf_counter() - T_START:7.1f} s] {msg}", file=sys.stderr, flush=True)


MAPS_ENV = "BENCH_MAPS_FILE"


def write_maps(tag):
    """/proc/self/maps of the measurement process into $BENCH_MAPS_FILE (or
    --profile-dir/bench_<pid>.maps), written when the GPU is first used and
    again after the line, so the raw PCs a fault handler prints at exit
    resolve to DSO + offset (tools/resolve_pcs.py).  Off without either."""
    path = os.environ.get(MAPS_ENV)
    if not path and PROFILE_DIR:
        path = os.path.join(PROFILE_DIR, f"bench_{os.getpid()}.maps")
    if not path:
        return
    try:
        with open("/proc/self/maps") as f, open(path, "w") as o:
            o.write(f"# {tag}, pid {os.getpid()}\n" + f.read())
    except OSError:
        pass


PROFILE_DIR = None


class LineState:
    """The line under construction in the measurement child (rank 0).  save()
    replaces the supervisor's state file atomically with the line so far, the
    leg running now (and the line key its result goes to) and whether the
    line is final."""

    def __init__(self, path):
        self.path = path
        self.line = None

    def save(self, running=None, key=None, final=False):
        if not self.path or self.line is None:
            return
        tmp = self.path + ".tmp"
        with open(tmp, "w") as f:
            json.dump({"line": self.line, "running": running, "running_key": key,
                       "final": final}, f)
        os.replace(tmp, self.path)


STATE = LineState(os.environ.get(STATE_ENV))


def wants_supervisor(args) -> bool:
    """Run as a script, the measurement goes to a child of a GPU-free parent,
    except: in the child itself, in the probe children, with --no-supervisor,
    under rocprofv3 (its preloaded library has already initialised the GPU
    in this process, so this process must not start another program: the
    profiled process itself is the measurement) and in the spawn launcher
    (each rank process it starts supervises its own child)."""
    if STATE.path or args.no_supervisor or args.traffic_probe or args.trace_probe:
        return False
    if under_rocprof():
        return False
    return not (args.gpus > 1 and "WORLD_SIZE" not in os.environ)


def exit_status(rc: int) -> str:
    """A child's return code as a shell reports it: `SIGSEGV` or `exit 3`."""
    import signal
    if rc < 0:
        try:
            return signal.Signals(-rc).name
        except ValueError:
            return f"signal {-rc}"
    return f"exit {rc}"


def shell_rc(rc: int) -> int:
    return rc if rc >= 0 else 128 - rc  # a signal (-N) becomes 128 + N


def supervise(argv) -> int:
    """The GPU-free parent: start the measurement child (`-X faulthandler`,
    same argv and environment, plus the state file's path), forward
    SIGTERM / SIGINT / SIGHUP to it, wait, and print its line."""
    import signal
    import tempfile
    fd, path = tempfile.mkstemp(prefix="bench_state_", suffix=".json")
    os.close(fd)
    os.unlink(path)  # the child creates it at its first checkpoint
    env = dict(os.environ, **{STATE_ENV: path})
    child = subprocess.Popen([sys.executable, "-X", "faulthandler", os.path.abspath(__file__)]
                             + list(argv), env=env)

    def forward(sig, _frame):
        try:
            child.send_signal(sig)
        except OSError:
            pass
    for sig in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP):
        signal.signal(sig, forward)
    rc = child.wait()
    st = None
    try:
        with open(path) as f:
            st = json.load(f)
    except (OSError, ValueError):
        pass
    finally:
        for p in (path, path + ".tmp"):
            try:
                os.unlink(p)
            except OSError:
                pass
    return finish_supervised(st, rc)


def finish_supervised(st, rc: int) -> int:
    """Print the child's line and return the bench's exit code.  A final line
    is printed as the child wrote it, with the child's code.  Otherwise the
    last checkpoint is printed with parity_check.aborted = "<leg>: <signal>"
    (or the exit code), all_ok false, the running leg's entry replaced by an
    error, and the exit code is non-zero.  Without any checkpoint (the child
    died before its timed region ended) there is no line."""
    if st is None or not st.get("line"):
        if rc != 0:
            progress(f"measurement child ended with {exit_status(rc)} before the timed region "
                     "was complete: no line")
        return shell_rc(rc)
    line = st["line"]
    if st.get("final"):
        if rc != 0 and rc != 1:  # died after writing a complete line (teardown)
            line.setdefault("parity_check", {})["aborted"] = f"after the line: {exit_status(rc)}"
            line["parity_check"]["all_ok"] = False
        emit(line)
        return shell_rc(rc)
    why = exit_status(rc) if rc != 0 else "exit 0 without a final line"
    leg = st.get("running")
    pc = line.setdefault("parity_check", {})
    pc["aborted"] = f"{leg or 'between legs'}: {why}"
    pc["all_ok"] = False
    if leg:
        pc.setdefault("failed", []).append(f"leg {leg}")
        if st.get("running_key"):
            line[st["running_key"]] = {"error": f"measurement child died in this leg: {why}"}
    progress(f"measurement child ended with {why} in leg {leg}: printing the line so far")
    emit(line)
    return shell_rc(rc) if rc != 0 else 1


# ---------------------------------------------------------------- launcher
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


RANK_GRACE_S = 10.0   # SIGTERM -> SIGKILL grace for the siblings of a failed rank
PG_TIMEOUT_S = 180.0  # process-group timeout (rendezvous and every collective)


def launch_ranks(args, argv=None) -> int:
    """--gpus N without torchrun: start N rank processes (this process never
    touches the GPU) and reap them in the order they exit (os.wait).  The
    first rank that exits non-zero ends the job: its siblings get SIGTERM,
    then SIGKILL after RANK_GRACE_S, and its exit code is returned with the
    rank named on stderr.  (Waiting on the ranks in rank order would leave the
    others blocked in a barrier until the process-group timeout.)  0 when
    every rank exits 0."""
    import signal
    port = _free_port()
    argv = sys.argv[1:] if argv is None else argv
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=JSON_OUT))  # rank 0's line on this stdout
    by_pid = {p.pid: (r, p) for r, p in enumerate(procs)}
    failed = None
    while by_pid and failed is None:
        pid, status = os.wait()  # the next rank to exit, in the order they exit
        if pid not in by_pid:
            continue
        r, p = by_pid.pop(pid)
        p.returncode = os.waitstatus_to_exitcode(status)
        if p.returncode != 0:
            failed = (r, p.returncode)
    if failed is None:
        return 0
    rank, rc = failed
    print(f"bench.py: rank {rank} exited {rc}; terminating the other ranks", file=sys.stderr,
          flush=True)
    live = [p for _, p in by_pid.values()]
    for p in live:
        p.send_signal(signal.SIGTERM)
    t_end = time.time() + RANK_GRACE_S
    for p in live:
        try:
            p.wait(timeout=max(0.0, t_end - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    return rc if rc > 0 else 128 - rc  # a signal (-N) becomes 128 + N, as a shell reports it


class Runtime:
    """Device, process group and clock of one rank (stub: CPU only)."""

    def __init__(self, args):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={self.world}")
        import torch
        self.torch = torch
        self.stub = args.stub
        self.stub_ordinal = 0 if args.one_device else self.local
        if self.stub:
            self.device = torch.device("cpu")
        else:
            self.device = torch.device("cuda", 0 if args.one_device else self.local)
            torch.cuda.set_device(self.device)
        self.dist = None
        if self.world > 1 or "TORCHELASTIC_RUN_ID" in os.environ:  # under torchrun: RCCL even at N=1
            import datetime
            import torch.distributed as dist
            kw = {"timeout": datetime.timedelta(seconds=PG_TIMEOUT_S)}
            if args.backend == "nccl":
                kw["device_id"] = self.device
            dist.init_process_group(args.backend, **kw)
            assert dist.get_world_size() == self.world == args.gpus
            self.dist = dist
        self.coll_device = "cpu" if args.backend == "gloo" else self.device
        if os.environ.get("BENCH_FAIL_RANK") == str(self.rank):
            # test hook (tests/test_parallel.py): this rank dies right after
            # joining the process group, as a rank that faults early would
            raise SystemExit(3)

    def device_info(self) -> dict:
        """This rank's device as the process sees it: the HIP ordinal and the
        PCI bus id (distinct ids per rank prove one GPU per rank)."""
        if self.stub:  # the ordinal the real run binds (cuda:LOCAL_RANK), for the launcher tests
            return {"rank": self.rank, "device": "cpu", "pci_bus_id": None,
                    "stub_ordinal": self.stub_ordinal}
        p = self.torch.cuda.get_device_properties(self.device)
        bus = getattr(p, "pci_bus_id", None)
        return {"rank": self.rank, "device": self.torch.cuda.current_device(),
                "pci_bus_id": bus, "name": p.name}

    def gather_objects(self, obj) -> list:
        if not self.dist:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def sync(self):
        if not self.stub:
            self.torch.cuda.synchronize()

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def gather_over_ranks(self, x: float) -> list:
        from bfrs import parallel
        return parallel.gather_over_ranks(x, self.dist, device=self.coll_device)

    def max_over_ranks(self, x: float) -> float:
        from bfrs import parallel
        return parallel.max_over_ranks(x, self.dist, device=self.coll_device)

    def observed_world(self) -> int:
        return self.dist.get_world_size() if self.dist else 1

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def timed(rt, step, steps):
    """K steps between barrier + synchronize on both sides; returns (this
    rank's seconds, max over ranks)."""
    rt.barrier()
    rt.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    rt.sync()
    el = time.perf_counter() - t0
    rt.barrier()
    return el, rt.max_over_ranks(el)


def device_loop(rt, step, stream, args):
    """Settle, W warmup steps, then the timed region: K steps between a
    barrier + synchronize on both sides.  HIP events on the launch stream
    bracket the same region: every launch in it is gf_apply (2 per step), so
    their mean duration = span / 2K.  Returns (settle steps, this rank's
    seconds, launch ms).  The bench and its kernel-trace child run this same
    loop, so the trace's last 2K dispatches are the child's timed region."""
    settle_steps = settle(rt, step, args.settle_ms)
    for _ in range(args.warmup):
        step()
    rt.sync()
    # (the correctness guard runs after the timed region: host work here would
    # idle the GPU and the timed region would start on ramping clocks again)
    torch = rt.torch
    if stream is not None:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    rt.barrier()
    rt.sync()
    t0 = time.perf_counter()
    if stream is not None:
        ev0.record(stream)
    for _ in range(args.steps):
        step()
    if stream is not None:
        ev1.record(stream)
    rt.sync()
    elapsed = time.perf_counter() - t0  # this rank's K steps; the job time is the max over ranks
    rt.barrier()
    launch_ms = ev0.elapsed_time(ev1) / (2 * args.steps) if stream is not None else None
    return settle_steps, elapsed, launch_ms


def settle(rt, step, ms):
    """Untimed steps for `ms` of wall time (clock ramp)."""
    n, t0 = 0, time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        step()
        n += 1
        if n % 16 == 0:
            rt.sync()
    rt.sync()
    return n


# ---------------------------------------------------------------- workloads
class ShardSets:
    """Data, parity and restored shard rows of one batch, rows
    bfrs_shard_pitch(S) apart, plus the pointer lists of one
    encode and one 3-erasure decode of every block."""

    def __init__(self, rt, shapes, S, layout="separate", pitch=-1):
        import numpy as np
        torch = rt.torch
        nseg, nb = sum(shapes), len(shapes)
        if rt.stub:
            pitch = S
        else:
            import bfrs
            pitch = bfrs.shard_pitch(S) if pitch < 0 else max(pitch, S)
        n_rows = {"data": nseg, "parity": 3 * nb, "restored": 3 * nb}
        sets, row0 = {}, 0
        if layout == "single":
            whole = torch.empty(sum(n_rows.values()) * pitch, dtype=torch.uint8, device=rt.device)
        for name, n in n_rows.items():
            if layout == "single":
                sets[name] = whole[row0 * pitch:].as_strided((n, S), (pitch, 1))
                row0 += n
            else:
                buf = torch.empty(n * pitch, dtype=torch.uint8, device=rt.device)
                sets[name] = buf.as_strided((n, S), (pitch, 1))
        self.shapes, self.S, self.pitch = shapes, S, pitch
        self.data, self.parity, self.restored = sets["data"], sets["parity"], sets["restored"]
        self.enc_in = [self.data[s] for s in range(nseg)]
        self.enc_out = [self.parity[i] for i in range(3 * nb)]
        self.dec_in, self.dec_out, self.erased = [], [], []
        seg = 0
        for b, k in enumerate(shapes):
            er = sorted(np.random.default_rng(0xDEC0DE + b).choice(k, min(3, k), replace=False).tolist())
            self.erased.append(er)
            for i in range(k):
                self.dec_in.append(None if i in er else self.data[seg + i])
                self.dec_out.append(self.restored[3 * b + er.index(i)] if i in er else None)
            seg += k

    def check_restored(self):
        seg = 0
        for b, k in enumerate(self.shapes):
            for t, i in enumerate(self.erased[b]):
                assert self.torch_equal(self.restored[3 * b + t], self.data[seg + i]), "decode mismatch"
            seg += k

    @staticmethod
    def torch_equal(a, b):
        import torch
        return torch.equal(a, b)


def codec_calls(rt, ctx, sets):
    """(encode(stream), decode(stream)) for the batch; stub: a stand-in that
    only touches the same buffers (launcher tests on CPU, never measured)."""
    if rt.stub:
        def enc(_h=None):
            off = 0
            for b, k in enumerate(sets.shapes):
                x = sets.data[off:off + k].sum(dim=0, dtype=rt.torch.uint8)
                for j in range(3):
                    sets.parity[3 * b + j].copy_(x + j)
                off += k

        def dec(_h=None):
            off = 0
            for b, k in enumerate(sets.shapes):
                for t, i in enumerate(sets.erased[b]):
                    sets.restored[3 * b + t].copy_(sets.data[off + i])
                off += k
        return enc, dec
    enc = ctx.prepare_encode(sets.shapes, 3, sets.S, sets.enc_in, sets.enc_out)
    dec = ctx.prepare_decode(sets.shapes, 3, sets.S, sets.dec_in, sets.enc_out, sets.dec_out)
    return enc, dec


def fill(rt, sets, seed, lo_b=0, S_full=None):
    """Synthetic splitmix64 bytes; with a stripe [lo_b, lo_b + S) of S_full-byte segments."""
    from bfrs import synth
    torch = rt.torch
    if S_full is None or S_full == sets.S:
        for s in range(sets.data.shape[0]):
            synth.fill_segment_torch(sets.data[s], seed, s)
        return
    row = torch.empty(S_full + 8, dtype=torch.uint8, device=rt.device)
    n8 = (S_full + 7) // 8 * 8
    for s in range(sets.data.shape[0]):
        synth.fill_segment_torch(row[:n8], seed, s)
        sets.data[s].copy_(row[lo_b:lo_b + sets.S])


def run_c4_strong(rt, ctx, args, stream_handle):
    """BASELINE configs[3]: one 320-segment job, rank g owns the 64-B-aligned
    column stripe g of every shard.  Encode and 3-erasure decode
    timed separately; GiB/s of the WHOLE job's original data."""
    from bfrs import parallel, synth
    S_full = args.segment_bytes
    shapes = synth.block_shapes(args.c4_segments)
    lo_b, hi_b = parallel.stripe_ranges(S_full, rt.world)[rt.rank]
    sets = ShardSets(rt, shapes, hi_b - lo_b, args.layout, -1)
    fill(rt, sets, 0xB10C, lo_b, S_full)
    enc, dec = codec_calls(rt, ctx, sets)
    steps = max(3, args.steps // 2)
    settle(rt, lambda: enc(stream_handle), min(args.settle_ms, 300.0))
    _, t_enc = timed(rt, lambda: enc(stream_handle), steps)
    settle(rt, lambda: dec(stream_handle), min(args.settle_ms, 300.0))
    _, t_dec = timed(rt, lambda: dec(stream_handle), steps)
    rt.sync()
    check = {"decode": check_restored(sets)}
    if rt.stub:
        check["encode"] = None
    elif rt.world == 1:
        check["encode"] = check_parity_golden(sets.parity, shapes, sets.S, 0xB10C, "c4_320x32MiB")
    else:
        check["encode"] = check_c4_stripes_golden(rt, sets.parity, shapes, S_full)
    pcie = None
    if args.pcie == "auto" and not rt.stub:
        # device-resident AND incl. pinned H2D/D2H; every
        # rank streams its own stripes over its own PCIe link
        pcie = pcie_inclusive(ctx, sets, steps=1, rt=rt, job_bytes=sum(shapes) * S_full)
        pcie["note"] = ("whole-job GiB/s, max over ranks; each rank's stripes from pinned host "
                        "buffers through bfrs_*_host_batch")
    if args.dump_dir:
        import numpy as np
        os.makedirs(args.dump_dir, exist_ok=True)
        np.save(os.path.join(args.dump_dir, f"c4_parity_rank{rt.rank}.npy"),
                sets.parity.cpu().numpy())
        with open(os.path.join(args.dump_dir, f"c4_stripe_rank{rt.rank}.json"), "w") as f:
            json.dump({"lo": lo_b, "hi": hi_b, "shapes": shapes, "segment_bytes": S_full}, f)
    job = sum(shapes) * S_full
    out = {
        "workload": "configs[3]: 320 x 32 MiB = 10xRS(30,3)+1xRS(20,3), 64-B column stripes over "
                    f"{rt.world} GPU(s)",
        "scaling": "strong", "blocks": shapes, "stripe_bytes_per_gpu": hi_b - lo_b,
        "steps": steps,
        "encode_GiBps": round(job * steps / 2**30 / t_enc, 2),
        "decode_GiBps": round(job * steps / 2**30 / t_dec, 2),
        "value": round(2 * job * steps / 2**30 / (t_enc + t_dec), 2),
        "unit": "GiB/s",
        "ms_per_encode": round(t_enc / steps * 1e3, 4), "ms_per_decode": round(t_dec / steps * 1e3, 4),
        "pcie_inclusive": pcie,
        "parity_check": check,
    }
    del sets
    return out


# ---------------------------------------------------------------- parity check
GOLDEN = os.path.join(ROOT, "tests", "golden", "rs_large.json")


def check_c4_stripes_golden(rt, parity, shapes, S_full):
    """N > 1: the golden digests cover whole shards, so after the timed region
    every rank's parity stripes are all-gathered (one collective, outside
    any timing), rank 0 reassembles the 33 whole shards and checks them
    against tests/golden/rs_large.json["c4_320x32MiB"]."""
    from bfrs import parallel
    torch = rt.torch
    ranges = parallel.stripe_ranges(S_full, rt.world)
    wmax = max(hi - lo for lo, hi in ranges)
    mine = torch.zeros(parity.shape[0], wmax, dtype=torch.uint8, device=rt.coll_device)
    mine[:, :parity.shape[1]].copy_(parity)
    parts = [torch.empty_like(mine) for _ in range(rt.world)]
    rt.dist.all_gather(parts, mine)
    if rt.rank != 0:
        return {"match": None, "note": "checked on rank 0"}
    whole = torch.empty(parity.shape[0], S_full, dtype=torch.uint8, device=rt.coll_device)
    for g, (lo, hi) in enumerate(ranges):
        whole[:, lo:hi].copy_(parts[g][:, :hi - lo])
    del parts
    r = check_parity_golden(whole, shapes, S_full, 0xB10C, "c4_320x32MiB")
    if r is not None:
        r["assembled_from_ranks"] = rt.world
    return r


def golden_parity(name):
    try:
        return json.load(open(GOLDEN))[name]
    except (OSError, ValueError, KeyError):
        return None


def check_parity_golden(parity_rows, shapes, S, seed, name):
    """SHA-256 of every parity shard the timed launches wrote against the
    committed oracle digests (tests/golden/rs_large.json[name]); None when no
    golden entry covers this batch (other sizes / seeds)."""
    import hashlib
    g = golden_parity(name)
    if not g or g["blocks"] != list(shapes) or g["segment_size"] != S or g["seed"] != seed:
        return None
    bad = []
    for b in range(len(shapes)):
        for j in range(3):
            h = hashlib.sha256(parity_rows[3 * b + j].cpu().numpy().tobytes()).hexdigest()
            if h != g["parity_sha256"][b][j]:
                bad.append([b, j])
    return {"golden": f"tests/golden/rs_large.json[{name}]", "shards": 3 * len(shapes),
            "mismatched": bad, "match": not bad}


def golden_covers(name, shapes, S, seed) -> bool:
    """True when tests/golden/rs_large.json[name] is the digest set of exactly
    this batch, so its check must run and must match."""
    g = golden_parity(name)
    return bool(g) and g["blocks"] == list(shapes) and g["segment_size"] == S and g["seed"] == seed


class Legs:
    """The side legs of a bench line (config 1, device BLAKE3, PCIe, crate
    API, CPU baseline, config 5).  Every exception becomes the leg's
    {"error": ...} entry, which parity_summary counts as a FAILED check: the
    line still prints, with all_ok false, and the process exits non-zero.
    OSError / MemoryError (disk space for c5's archive, host memory for
    pinned buffers) let the later legs run; anything else (a BfrsError from
    the library, a HIP fault, a wrong result) skips them, since the device
    may be unusable, and names the leg in parity_check.aborted."""

    def __init__(self):
        self.aborted = None

    def run(self, name, fn, *a):
        if self.aborted:
            return {"error": f"skipped: {self.aborted}"}
        progress(f"leg {name}")
        try:
            return fn(*a)
        except (OSError, MemoryError) as e:
            return {"error": f"{type(e).__name__}: {e}"}
        except Exception as e:  # noqa: BLE001 - recorded as this leg's failure
            self.aborted = f"{name} raised {type(e).__name__}"
            return {"error": f"{type(e).__name__}: {e}"}


def leg_flag(res, *path):
    """The check value at `path` inside an enabled leg's result; a missing
    result or an {"error": ...} entry is a failed check (False), never None."""
    if not isinstance(res, dict) or "error" in res:
        return False
    v = res
    for k in path:
        v = v.get(k) if isinstance(v, dict) else None
    return v


def parity_summary(enabled, detail):
    """parity_check of the line: `enabled` maps each check to (expected?,
    value).  An expected check passes only with value True: False, None (the
    check did not run) and an error entry all fail, so all_ok cannot be true
    while an enabled check was skipped.  Checks that do not apply (no golden
    covers a non-default batch size, a leg switched off) are listed apart."""
    failed = [k for k, (exp, v) in enabled.items() if exp and v is not True]
    out = dict(detail)
    out["expected"] = sorted(k for k, (exp, _) in enabled.items() if exp)
    out["not_applicable"] = sorted(k for k, (exp, _) in enabled.items() if not exp)
    out["failed"] = failed
    out["all_ok"] = not failed
    return out


def check_restored(sets):
    """The restored shards of the timed decodes equal the erased originals."""
    seg, bad = 0, []
    for b, k in enumerate(sets.shapes):
        for t, i in enumerate(sets.erased[b]):
            if not sets.torch_equal(sets.restored[3 * b + t], sets.data[seg + i]):
                bad.append([b, i])
        seg += k
    return {"restored_shards": sum(len(e) for e in sets.erased), "mismatched": bad, "match": not bad}


def c4_one_process(args, ctx, world, one_device=False, steps=2):
    """c4_strong.pcie_inclusive_one_process: BASELINE configs[3] (320 x 32 MiB)
    from pinned host memory through bfrs_encode_host_batch_multi /
    bfrs_decode_host_batch_multi, ONE process driving one context per GPU
    (BlockFrame is one process, commit.rs:391-393), beside the one-process-
    per-GPU figure (c4_strong.pcie_inclusive).  Rank 0 runs it after the
    other ranks have left their devices.  Parity checked against the golden
    digests, restored shards against the originals."""
    import torch
    import bfrs
    from bfrs import synth
    S = args.segment_bytes
    shapes = synth.block_shapes(args.c4_segments)
    nseg, nb = sum(shapes), len(shapes)
    host = torch.empty(nseg, S, dtype=torch.uint8, pin_memory=True)
    row = torch.empty(S + 8, dtype=torch.uint8, device=f"cuda:{ctx.device}")
    n8 = (S + 7) // 8 * 8
    for s in range(nseg):
        synth.fill_segment_torch(row[:n8], 0xB10C, s)
        host[s].copy_(row[:S])
    del row
    par = torch.empty(3 * nb, S, dtype=torch.uint8, pin_memory=True)
    rest = torch.empty(3 * nb, S, dtype=torch.uint8, pin_memory=True)
    import numpy as np
    enc_in = [host[s] for s in range(nseg)]
    enc_out = [par[i] for i in range(3 * nb)]
    dec_in, dec_out, want, seg = [], [], [], 0
    for b, k in enumerate(shapes):
        er = sorted(np.random.default_rng(0xDEC0DE + b).choice(k, min(3, k), replace=False).tolist())
        for i in range(k):
            dec_in.append(None if i in er else host[seg + i])
            dec_out.append(rest[3 * b + er.index(i)] if i in er else None)
            if i in er:
                want.append((3 * b + er.index(i), seg + i))
        seg += k
    # one context per GPU this process can see (under a launcher that hides
    # the other ranks' devices it falls back to the visible ones)
    visible = torch.cuda.device_count()
    devs = [0] * (world - 1) if one_device else [d for d in range(world) if d != ctx.device][:max(0, min(world, visible) - 1)]
    extra = [bfrs.Context(d) for d in devs]
    ctxs = [ctx] + extra
    try:
        def clock(call):
            call()  # warm: pins nothing new, grows each context's slab buffers
            t0 = time.perf_counter()
            for _ in range(steps):
                call()
            return (time.perf_counter() - t0) / steps
        t_enc = clock(lambda: bfrs.encode_host_batch_multi(ctxs, shapes, 3, S, enc_in, enc_out))
        t_dec = clock(lambda: bfrs.decode_host_batch_multi(ctxs, shapes, 3, S, dec_in, enc_out,
                                                           dec_out))
    finally:
        for c in extra:
            c.close()
    golden = check_parity_golden(par, shapes, S, 0xB10C, "c4_320x32MiB")
    restored_ok = all(torch.equal(rest[r], host[s]) for r, s in want)
    gib = nseg * S / 2**30
    del host, par, rest
    return {
        "contexts": len(ctxs), "devices": sorted({ctx.device} | set(devs)),
        "contexts_on_device_0": one_device or world == 1,
        "encode_GiBps": round(gib / t_enc, 2), "decode_GiBps": round(gib / t_dec, 2),
        "encode_ms": round(t_enc * 1e3, 2), "decode_ms": round(t_dec * 1e3, 2),
        "parity_golden": golden, "restored_match": restored_ok,
        "match": bool(restored_ok and (golden or {}).get("match") is not False
                      and (golden is not None or S != 32 << 20 or args.c4_segments != 320)),
        "what": "one process, one context per GPU: bfrs_*_host_batch_multi over pinned host "
                "buffers (context d = column stripe d of every shard); whole-job GiB/s, mean "
                f"of {steps} timed calls after a warm call",
    }


def traffic_probe(args):
    """--traffic-probe: the child process of one live PMC pass.  The bench's
    C2 batch (same shapes, pitch, layout, seed), 3 encode + 3 decode launches,
    nothing timed; rocprofv3 counts every dispatch."""
    from bfrs import synth
    import bfrs
    rt = Runtime(args)
    sets = ShardSets(rt, synth.block_shapes(args.segments), args.segment_bytes, args.layout,
                     args.pitch)
    fill(rt, sets, 0xB10C)
    ctx = bfrs.Context(rt.device.index)
    enc, dec = codec_calls(rt, ctx, sets)
    sh = rt.torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        enc(sh)
        dec(sh)
    rt.sync()
    return 0


def per_launch_events(rt, encode, decode, stream, sh, steps, settle_ms=300.0):
    """Every launch's own duration in THIS process, without a profiler: after
    `settle_ms` of settle steps on the timed region's buffers, K more steps
    with a pair of HIP events on the launch stream around each launch (the
    events sit between launches, so each pair brackets one gf_apply kernel).
    Returns mean / median / min / max over the 2K launches, or {"error": ...}.
    (Round 4 read the same figures from torch's profiler; a second profiler
    session in one process is the prime suspect of round 4's SIGSEGV, so no
    profiler runs in the bench process any more: DESIGN.md §5.)"""
    import statistics
    torch = rt.torch
    try:
        settle(rt, lambda: (encode(sh), decode(sh)), settle_ms)
        pairs = []
        for _ in range(steps):
            for fn in (encode, decode):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                fn(sh)
                b.record(stream)
                pairs.append((a, b))
        torch.cuda.synchronize()
        d = [a.elapsed_time(b) for a, b in pairs]
        return {"how": f"HIP event pair around each of {len(d)} launches (K steps after "
                       f"{settle_ms:.0f} ms of settle steps, same process and buffers as the "
                       "timed region)",
                "launches": len(d), "mean_ms": round(statistics.mean(d), 4),
                "median_ms": round(statistics.median(d), 4), "min_ms": round(min(d), 4),
                "max_ms": round(max(d), 4)}
    except Exception as e:  # noqa: BLE001 - informative only
        return {"error": f"{type(e).__name__}: {e}"}


def trace_probe(args):
    """--trace-probe: the child of the live kernel-trace pass.  The bench's
    own device part, unchanged: the same C2 batch (shapes, pitch, layout,
    seed, allocation order), the same settle / warmup / timed loop
    (device_loop), so rocprofv3 times the same kind of launches the line's
    HIP events time.  Prints its own event launch_ms as a JSON line."""
    from bfrs import synth
    import bfrs
    rt = Runtime(args)
    sets = ShardSets(rt, synth.block_shapes(args.segments), args.segment_bytes, args.layout,
                     args.pitch)
    fill(rt, sets, 0xB10C)
    ctx = bfrs.Context(rt.device.index)
    enc, dec = codec_calls(rt, ctx, sets)
    stream = rt.torch.cuda.current_stream()
    sh = stream.cuda_stream

    def step():
        enc(sh)
        dec(sh)
    _, elapsed, launch_ms = device_loop(rt, step, stream, args)
    # then the device BLAKE3 of the 128 data segments, as blake3_device calls it
    call, digests = ctx.blake3_batch_dev_call([sets.data[i] for i in range(sets.data.shape[0])])
    for _ in range(B3_PROBE_CALLS):
        call()
    rt.sync()
    emit({"launch_ms": launch_ms, "steps": args.steps, "ms_per_step": elapsed / args.steps * 1e3,
          "blake3_calls": B3_PROBE_CALLS, "blake3_digest0": bytes(digests[0]).hex()})
    return 0


def main(argv=None):
    args = parse(argv)
    if args.stub_legs_builtin:
        globals().update(stub_leg_standins())
    if args.workload == "c5":
        line = run_c5(args)
        line.update({"n_gpus": 1, "higher_is_better": True, "vs_baseline": None, "dtype": "u8",
                     "data": "synthetic splitmix64 bytes; files in the page cache"})
        emit(line)
        return 0 if line["blake3_match"] else 1
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args, argv)
    if args.traffic_probe:
        return traffic_probe(args)
    if args.trace_probe:
        return trace_probe(args)
    solo = (args.gpus == 1 and not args.stub and not args.strong
            and int(os.environ.get("WORLD_SIZE", "1")) == 1 and not under_rocprof())
    live_traffic = live_trace = None
    if args.pmc == "auto" and solo:
        # before anything in this process touches the GPU: the passes are child processes
        live_traffic = live_pmc_traffic(args)
        progress("live PMC passes done")
    if args.trace == "auto" and solo:
        live_trace = live_kernel_trace(args, args.profile_dir)
        progress("live kernel-trace pass done")
    rayon_child = None
    if args.crate == "auto" and solo:
        rayon_child = rayon_fresh_process()  # a child process too, before the GPU is touched
        progress("rayon child done")
    from bfrs import parallel, synth

    rt = Runtime(args)
    torch = rt.torch
    global PROFILE_DIR
    PROFILE_DIR = args.profile_dir
    S_full = args.segment_bytes
    shapes = synth.block_shapes(args.segments)
    if args.strong:  # value = C4: this rank's 64-B column stripe of every shard
        lo_b, hi_b = parallel.stripe_ranges(S_full, rt.world)[rt.rank]
        S, seed = hi_b - lo_b, 0xB10C
    else:
        # every rank encodes the golden batch (seed 0xB10C, tests/golden/
        # rs_large.json): each GPU computes its own copy, so each can be
        # checked bit-exact against the committed digests after the timed region
        lo_b, S, seed = 0, S_full, 0xB10C
    sets = ShardSets(rt, shapes, S, args.layout, args.pitch)
    fill(rt, sets, seed, lo_b, S_full)

    ctx = stream = None
    if not rt.stub:
        import bfrs
        # crate_api runs one codec object per C2 block on as many threads (as
        # rayon does): let the context keep that many idle codec slots
        # (include/bfrs.h; the library default is 2)
        os.environ.setdefault("BFRS_CODEC_SLOTS", "8")
        ctx = bfrs.Context(rt.device.index)
        write_maps("after bfrs_open")
        stream = torch.cuda.current_stream()
        sh = stream.cuda_stream
    else:
        sh = None
    encode, decode = codec_calls(rt, ctx, sets)

    def step():
        encode(sh)
        decode(sh)

    settle_steps, elapsed, launch_ms = device_loop(rt, step, stream, args)
    if rt.rank == 0:
        progress("timed region done")
    rank_ms = [round(x / args.steps * 1e3, 4) for x in rt.gather_over_ranks(elapsed)]
    elapsed = rt.max_over_ranks(elapsed)

    enc_ms = dec_ms = copy_ms = events = None
    if not rt.stub:
        # Per-direction rates: short back-to-back loops after the timed region.
        def per_launch(fn, n=max(3, args.steps // 2)):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for _ in range(n):
                fn(sh)
            b.record(stream)
            torch.cuda.synchronize()
            return a.elapsed_time(b) / n
        enc_ms, dec_ms = per_launch(encode), per_launch(decode)
        # every launch's own duration in this process (HIP event pairs; no profiler)
        events = per_launch_events(rt, encode, decode, stream, sh, args.steps)
        # reference point on this box: a plain device copy (torch copy_) moving the
        # same read + write bytes as one gf_apply launch (SURVEY 8(d) "achievable")
        alg_bytes_launch = sum(k + 3 for k in shapes) * S
        cp_src = torch.empty(alg_bytes_launch // 2, dtype=torch.uint8, device=rt.device)
        cp_dst = torch.empty_like(cp_src)
        copy_ms = per_launch(lambda _h: cp_dst.copy_(cp_src))
        del cp_src, cp_dst
    rt.sync()
    # correctness of the measured buffers: every rank's parity against the
    # golden digests, every rank's restored shards against its originals
    my_check = {"encode": (check_parity_golden(sets.parity, shapes, S, seed, "c2_128x32MiB")
                           if not rt.stub else None),
                "decode": check_restored(sets)}
    ok_here = my_check["decode"]["match"] and (my_check["encode"] or {}).get("match") is not False
    ranks_ok = rt.gather_over_ranks(1.0 if ok_here else 0.0)
    data_bytes = sum(shapes) * S                     # original data per direction (this rank)
    alg_bytes = sum(k + 3 for k in shapes) * S        # HBM bytes per launch (both directions)
    scaling = "strong" if args.strong else "weak"
    job_bytes_step = 2 * sum(shapes) * (S_full if args.strong else S)
    value = parallel.throughput(job_bytes_step, rt.world, args.steps, elapsed, scaling)

    n1 = rt.world == 1
    real = not rt.stub or args.stub_legs  # --stub-legs: the CPU tests' stand-ins run the legs
    solo_legs = n1 and real and not args.strong
    golden_c2 = golden_covers("c2_128x32MiB", shapes, S, seed) and not rt.stub
    golden_c4 = (golden_covers("c4_320x32MiB", synth.block_shapes(args.c4_segments), S_full, 0xB10C)
                 and not rt.stub)
    R = {}  # leg results by leg name

    line = None
    if rt.rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": rt.world,
            "world_size_observed": rt.observed_world(),
            "steps": args.steps,
            "warmup": args.warmup,
            "settle": {"ms": args.settle_ms, "steps": settle_steps,
                       "note": "untimed clock-settle steps before the warmup"},
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "rank_ms_per_step": rank_ms,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": ("STUB (CPU rehearsal of the launcher, not a measurement)" if rt.stub else
                     "synthetic splitmix64 bytes (seed 0xB10C on every rank), resident in HBM"),
            "config": {
                "workload": ("BASELINE configs[3]: 10 GiB archive, 320 x 32 MiB segments = "
                             "10xRS(30,3)+1xRS(20,3), column-striped over the GPUs"
                             if args.strong else
                             "BASELINE configs[1]+[2]: 128 x 32 MiB segments = 4xRS(30,3)+1xRS(8,3); "
                             "step = encode batch + 3-erasure decode of every block"),
                "segments": args.segments, "segment_bytes": S_full,
                "shard_pitch": int(sets_pitch(S, args, rt)),
                "layout": args.layout, "blocks": shapes, "parity_shards": 3,
                "parallelism": (f"64-B column stripes x{rt.world}" if args.strong
                                else f"independent batch per GPU x{rt.world}"),
                "kernel_variant": os.environ.get("BFRS_KERNEL_VARIANT", "default"),
            },
        }
        if not rt.stub:
            line["encode_GiBps_per_gpu"] = round(data_bytes / 2**30 / (enc_ms * 1e-3), 2)
            line["decode_GiBps_per_gpu"] = round(data_bytes / 2**30 / (dec_ms * 1e-3), 2)
            line["roofline"] = roofline(alg_bytes, launch_ms, enc_ms, dec_ms, copy_ms,
                                        live_traffic, live_trace, events)
        STATE.line = line

    def refresh():
        """parity_check of the line from the checks and legs done so far."""
        c4 = line.get("c4_strong")
        c4_pc = (c4 or {}).get("parity_check") or {}
        c1, b3, pcie, crate, cpu, c4_1p, c5 = (R.get(k) for k in (
            "c1_rs13", "blake3_device", "pcie_inclusive", "crate_api", "cpu_baseline",
            "c4_one_process", "c5"))
        legs_enabled = {
            "ranks_ok": (True, all(ranks_ok)),
            "c2_encode": (golden_c2, leg_flag(my_check["encode"], "match")),
            "c3_decode": (True, leg_flag(my_check["decode"], "match")),
            "c1_rs13": (real, leg_flag(c1, "match")),
            "c4_encode": (args.c4 == "auto" and not args.strong and golden_c4,
                          leg_flag(c4_pc.get("encode"), "match")),
            "c4_decode": (args.c4 == "auto" and not args.strong,
                          leg_flag(c4_pc.get("decode"), "match")),
            "c4_one_process": (real and args.c4 == "auto" and args.pcie == "auto" and not args.strong,
                               leg_flag(c4_1p, "match")),
            "c5_blake3": (solo_legs and args.c5 == "auto", leg_flag(c5, "blake3_match")),
            "c5_repair": (solo_legs and args.c5 == "auto", leg_flag(c5, "repair", "match")),
            "blake3_c2": (solo_legs and (golden_c2 or args.stub_legs),
                          leg_flag(b3, "parity_check", "match")),
            "blake3_device_ran": (solo_legs, isinstance(b3, dict) and "error" not in b3),
            "pcie_decode": (solo_legs and args.pcie == "auto", leg_flag(pcie, "decode_match")),
            "crate_recover": (solo_legs and args.crate == "auto", leg_flag(crate, "recover_match")),
            "cpu_baseline_self_check": (solo_legs and args.cpu_baseline == "auto",
                                        leg_flag(cpu, "self_check")),
        }
        line["parity_check"] = parity_summary(legs_enabled, {
            "c1_rs13": c1, "c2_encode": my_check["encode"], "c3_decode": my_check["decode"],
            "ranks_ok": [bool(x) for x in ranks_ok],
            "c4_encode": c4_pc.get("encode"), "c4_decode": c4_pc.get("decode"),
            "c5_blake3": None if c5 is None else c5.get("blake3_match"),
            "c5_repair": ((c5 or {}).get("repair") or {}).get("match"),
            "blake3_c2": ((b3 or {}).get("parity_check") or {}).get("match"),
            "when": "after the timed region, on the buffers the timed launches wrote"})
        if legs.aborted:
            line["parity_check"]["aborted"] = legs.aborted

    legs = Legs()
    if line is not None:
        refresh()
        STATE.save()  # the headline survives anything that follows

    c4 = None
    if args.c4 == "auto" and not args.strong:
        c4 = run_c4_strong(rt, ctx, args, sh)  # collective inside: every rank runs it, no guard
    devices = rt.gather_objects(rt.device_info())  # collective: every rank, before rank 0 goes on
    if rt.rank != 0:
        rt.sync()
        if ctx is not None:
            ctx.close()
        rt.close()
        return 0 if ok_here else 3
    line["c4_strong"] = c4
    line["rank_devices"] = devices
    line["host_budget"] = host_budget(args, rt.world)
    refresh()
    STATE.save()

    def leg(name, key, fn, *a):
        """One side leg, checkpointed before and after (the supervisor names
        the leg if the process dies inside it)."""
        STATE.save(running=name, key=key)
        if args.stub_crash_leg == name:  # test hook: the process dies inside this leg
            import signal
            os.kill(os.getpid(), signal.SIGSEGV)
        r = legs.run(name, fn, *a)
        R[name] = r
        if key:
            line[key] = r
        refresh()
        STATE.save()
        return r

    info = host_info()
    if real:
        leg("c1_rs13", None, check_config1, ctx)
    if solo_legs:
        b3 = leg("blake3_device", "blake3_device", blake3_device, ctx, sets)
        if isinstance(b3, dict) and "error" not in b3 and live_trace:
            b3["kernels"] = blake3_trace_figures(live_trace, b3["bytes"])
            STATE.save()
    if solo_legs and args.pcie == "auto":
        leg("pcie_inclusive", "pcie_inclusive", pcie_inclusive, ctx, sets)
    if solo_legs and args.crate == "auto":
        host_pinned = pinned_host_state(rt)
        if not rt.stub:
            # The earlier legs leave ~27 GB of pinned blocks in torch's caching
            # host allocator.  Held, they slowed the five concurrent blocks by
            # ~20% (r04ec: 85.4/87.4 ms emptied against 104.8/102.0 ms held, one
            # box, alternating).  A BlockFrame process holds no
            # such memory, so give it back first
            rt.torch._C._host_emptyCache()
            host_pinned["after_empty_cache"] = pinned_host_state(rt)
        load_before = host_pressure()
        crate = leg("crate_api", "crate_api", crate_api, ctx, sets)
        if isinstance(crate, dict) and "error" not in crate:
            crate["pinned_host_before"] = host_pinned
            crate["host_pressure"] = {"before": load_before, "after": host_pressure()}
            if rayon_child is not None:
                crate["generate_parity_all_blocks_fresh_process"] = rayon_child
            STATE.save()
    if solo_legs and args.cpu_baseline == "auto":
        leg("cpu_baseline", "cpu_baseline", cpu_baseline, args, sets, info)
    del sets
    if real and args.c4 == "auto" and args.pcie == "auto" and not args.strong:
        c4_1p = leg("c4_one_process", None, c4_one_process, args, ctx, rt.world, args.one_device)
        if c4 is not None:
            c4["pcie_inclusive_one_process"] = c4_1p
    if solo_legs and args.c5 == "auto":
        leg("c5", "c5", run_c5, args, ctx)
    if not rt.stub:
        for key in ("cpu_baseline", "crate_api", "pcie_inclusive", "c5", "blake3_device"):
            line.setdefault(key, None)
    refresh()
    emit(line)
    # ordered teardown: the device idle, the context
    # closed, then the process group; what is left goes through the binding's
    # atexit close (bfrs.close_all) before the runtimes' own teardown
    rt.sync()
    if ctx is not None:
        ctx.close()
    rt.close()
    write_maps("after the line")
    return 0 if line["parity_check"]["all_ok"] else 1


def roofline(alg_bytes, launch_ms, enc_ms, dec_ms, copy_ms, live_traffic, live_trace, events):
    """The line's roofline object: achieved = algorithmic bytes per launch /
    the launch time from HIP events over the timed region; traffic from the
    live PMC passes (or the committed record); the rocprofv3 child pass's
    kernel trace and this process's per-launch event pairs beside it."""
    achieved = alg_bytes / (launch_ms * 1e-3) / 1e9
    traffic, traffic_src = live_traffic if live_traffic else (None, None)
    if traffic is not None:
        traffic_src["ratio_to_algorithmic"] = round(traffic / alg_bytes, 4)
    else:
        live_err = (traffic_src or {}).get("error")
        traffic, traffic_src = pmc_traffic(alg_bytes)
        live_note = live_err or ("skipped under rocprofv3" if under_rocprof() else "off")
        traffic_src = dict(traffic_src or {}, live_pass=live_note)
    trace = live_trace
    if trace and "error" not in trace:
        trace = dict(trace)
        trace.pop("blake3", None)
        trace["ratio_mean_to_launch_ms"] = round(trace["mean_ms"] / launch_ms, 4)
        trace["frac_at_trace_mean"] = round(
            alg_bytes / (trace["mean_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
        trace["note"] = ("another process: its shard buffers land wherever the driver places "
                         "them, in either HBM placement mode (DESIGN.md §9b), so its launch "
                         "time can differ from this process's by the mode gap (~8%)")
    elif trace is None:
        trace = {"live_pass": "skipped under rocprofv3" if under_rocprof() else "off"}
    if events and "error" not in events:
        events["ratio_mean_to_launch_ms"] = round(events["mean_ms"] / launch_ms, 4)
        events["frac_at_mean"] = round(alg_bytes / (events["mean_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
    return {
        "bound": "hbm",
        "kernel": ("gf_apply_unrolled_kernel (variant 76: unrolled SDWA-addressed GF(2^8)-"
                   "subfield pass, contiguous-line nt loads)"
                   if os.environ.get("BFRS_KERNEL_VARIANT", "76") == "76" else
                   f"gf_apply (variant {os.environ.get('BFRS_KERNEL_VARIANT')})"),
        "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
        "traffic_source": traffic_src,
        "alg_bytes_per_launch": alg_bytes,
        "launch_ms": round(launch_ms, 4),
        "launch_ms_by_direction": {"encode": round(enc_ms, 4), "decode": round(dec_ms, 4)},
        "timing": "HIP events on the launch stream over the timed region / launches",
        "trace": trace,
        "per_launch_events": events,
        "device_copy_reference": {
            "GBps": round(alg_bytes / (copy_ms * 1e-3) / 1e9, 1),
            "ms": round(copy_ms, 4),
            "what": "torch copy_ of alg_bytes/2 bytes (same read + write bytes as one launch), same box"},
    }


def sets_pitch(S, args, rt):
    if rt.stub:
        return S
    import bfrs
    return bfrs.shard_pitch(S) if args.pitch < 0 else max(args.pitch, S)


if __name__ == "__main__":
    faulthandler.enable(all_threads=True)  # a fault prints every thread's Python stack
    claim_stdout()
    if wants_supervisor(parse()):
        sys.exit(supervise(sys.argv[1:]))
    # The measurement child exits through the interpreter's normal teardown
    # (round 5 left through os._exit after its line): a
    # fault there now reaches the supervisor's "after the line" check.
    sys.exit(main())

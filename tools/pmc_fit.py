"""Does a rocprofv3 --pmc counter set fit ONE pass?

rocprofv3 does not split counters over passes.  Per pass the hardware offers
at most 8 SQ_, 4 TCC_, 4 TCP_, 2 TA_, 2 TD_ and 2 GRBM_ counters
(MI355X_MICROARCH.md, rocprofv3 section); FETCH_SIZE takes 3 TCC slots and
WRITE_SIZE 2; the _sum / _avr / _min / _max forms of one counter and its
non-reduced per-instance form count once.  A set that asks for more makes
rocprofv3 print "error code 38: Request exceeds the capabilities of the
hardware to collect" and then hang, SIGTERM included -- the round-3
per-channel TCC pass hung exactly so at profiler start.

usage: python tools/pmc_fit.py COUNTER [COUNTER ...]   (exit 1 if it does not fit)
"""
import sys

LIMITS = {"SQ": 8, "TCC": 4, "TCP": 4, "TA": 2, "TD": 2, "GRBM": 2}
# derived counters and the hardware slots they take
DERIVED = {"FETCH_SIZE": {"TCC": 3}, "WRITE_SIZE": {"TCC": 2}}
REDUCTIONS = ("_sum", "_avr", "_min", "_max")


def base_name(counter: str) -> str:
    c = counter.split("[", 1)[0]  # per-instance form, e.g. TCC_REQ[3]
    for r in REDUCTIONS:
        if c.endswith(r):
            return c[: -len(r)]
    return c


def slots(counters):
    """{block: slots used} of a counter set."""
    used, seen = {}, set()
    for c in counters:
        b = base_name(c)
        if b in seen:
            continue
        seen.add(b)
        if b in DERIVED:
            for blk, n in DERIVED[b].items():
                used[blk] = used.get(blk, 0) + n
            continue
        blk = b.split("_", 1)[0]
        used[blk] = used.get(blk, 0) + 1
    return used


def problems(counters):
    """The blocks a set overfills, as messages (empty: it fits one pass)."""
    out = []
    for blk, n in sorted(slots(counters).items()):
        lim = LIMITS.get(blk)
        if lim is None:
            out.append(f"{blk}: unknown counter block (no per-pass limit on record)")
        elif n > lim:
            out.append(f"{blk}: {n} counters, one pass holds {lim}")
    return out


def main(argv):
    counters = [c for a in argv for c in a.split()]
    bad = problems(counters)
    if bad:
        print("pmc_fit: counter set does not fit one rocprofv3 pass: " + "; ".join(bad),
              file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))

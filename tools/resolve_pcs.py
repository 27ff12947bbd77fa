"""Resolve the raw PCs of a fault handler's stack ("@ 0x7f... (unknown)",
glog / rocprofv3 style, or faulthandler's) to DSO + offset with a
/proc/<pid>/maps dump of the same process (tools/teardown_probe.py,
tools/soak.py --maps).

usage: python tools/resolve_pcs.py stack.txt process.maps"""
import re
import sys


def load_maps(path):
    spans = []
    for line in open(path):
        m = re.match(r"([0-9a-f]+)-([0-9a-f]+) (\S+) ([0-9a-f]+) \S+ \d+\s*(.*)", line)
        if m:
            lo, hi, perms, off, name = m.groups()
            spans.append((int(lo, 16), int(hi, 16), perms, int(off, 16), name.strip() or "[anon]"))
    return spans


def resolve(pc, spans):
    for lo, hi, perms, off, name in spans:
        if lo <= pc < hi:
            return f"{name} +0x{pc - lo + off:x} ({perms})"
    return "(not mapped in this dump)"


def main(stack, maps):
    spans = load_maps(maps)
    for line in open(stack):
        for h in re.findall(r"0x[0-9a-f]{6,}", line):
            print(f"{h}  {resolve(int(h, 16), spans)}    <- {line.strip()[:80]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])

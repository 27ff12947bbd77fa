"""Per-kernel instruction mix of a hipcc --cuda-device-only -S listing.

usage: python tools/isa_stats.py kernels.s [substring]
"""
import re
import sys
from collections import Counter


def kernels(src):
    for m in re.finditer(r"^(_Z\S+):[^\n]*$", src, re.M):
        name = m.group(1)
        body = src[m.end():]
        end = body.find("s_endpgm")
        yield name, body[: end + 8]


def main():
    src = open(sys.argv[1]).read()
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    meta = dict(re.findall(r"\.name:\s+(\S+)\n(?:[^\n]*\n){0,60}?\s+\.vgpr_count:\s+(\d+)", src))
    for name, body in kernels(src):
        if pat not in name:
            continue
        ops = []
        for line in body.splitlines():
            t = line.strip()
            if not t or t.startswith((".", ";")) or t.endswith(":"):
                continue
            ops.append(t.split()[0])
        c = Counter(ops)
        valu = sum(n for o, n in c.items() if o.startswith("v_"))
        ds = sum(n for o, n in c.items() if o.startswith("ds_read"))
        print(f"{name[:70]}  vgpr={meta.get(name, '?')} valu={valu} ds_read={ds} "
              f"waitcnt={c['s_waitcnt']}")
        print("   ", c.most_common(14))


if __name__ == "__main__":
    main()

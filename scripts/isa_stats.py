"""Per-kernel register / scratch / occupancy table of a device assembly file.

    hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S -o x.s <file.hip> ...
    python scripts/isa_stats.py x.s [name-filter]
"""
import re
import subprocess
import sys


def main(path, filt=""):
    cur, rows = None, []
    stats = {}
    for line in open(path):
        m = re.match(r"^(_Z\w+):\s*;\s*@", line)
        if m:
            cur = m.group(1)
            stats = {}
            continue
        m = re.match(r"^; (NumVgprs|NumAgprs|TotalNumVgprs|ScratchSize|Occupancy|LDSByteSize): (\d+)", line)
        if m and cur:
            stats[m.group(1)] = int(m.group(2))
            if m.group(1) == "Occupancy":
                rows.append((cur, dict(stats)))
                cur = None
    names = subprocess.run(["c++filt"], input="\n".join(r[0] for r in rows), text=True,
                           capture_output=True).stdout.splitlines()
    for (sym, st), name in zip(rows, names):
        if filt in name:
            print(f"vgpr {st.get('NumVgprs', 0):3d} agpr {st.get('NumAgprs', 0):3d} "
                  f"scratch {st.get('ScratchSize', 0):4d} occ {st.get('Occupancy', 0)}  {name[:150]}")


if __name__ == "__main__":
    main(*sys.argv[1:])

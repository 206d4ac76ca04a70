"""Attribute the PCs of a crash trace to the DSOs of the process's memory map.

    python tools/resolve_pcs.py CRASH_LOG MAPS_FILE

CRASH_LOG holds glog-style frames ("@ 0x7f... (unknown)"), MAPS_FILE the /proc/self/maps
the same process wrote (bench.py with BENCH_EXIT_MAPS).  Prints, per frame, the DSO, the
offset into it and, when the DSO is readable here, the nearest dynamic symbol (nm -D).
"""
import bisect
import os
import re
import subprocess
import sys


def load_maps(path):
    segs = []
    for line in open(path):
        parts = line.split()
        if len(parts) < 6:
            continue
        lo, hi = (int(x, 16) for x in parts[0].split("-"))
        off = int(parts[2], 16)
        segs.append((lo, hi, off, parts[5]))
    segs.sort()
    return segs


def symbols(dso):
    try:
        out = subprocess.run(["nm", "-D", "--defined-only", dso], capture_output=True,
                             text=True, timeout=60).stdout
    except (OSError, subprocess.SubprocessError):
        return []
    syms = []
    for line in out.splitlines():
        p = line.split()
        if len(p) == 3:
            syms.append((int(p[0], 16), p[2]))
    syms.sort()
    return syms


def main():
    crash, maps = sys.argv[1:3]
    segs = load_maps(maps)
    starts = [s[0] for s in segs]
    cache = {}
    for line in open(crash):
        m = re.search(r"@\s+(0x[0-9a-f]+)|PC: @\s+(0x[0-9a-f]+)", line)
        if not m:
            continue
        pc = int(m.group(1) or m.group(2), 16)
        i = bisect.bisect_right(starts, pc) - 1
        if i < 0 or pc >= segs[i][1]:
            print(f"{pc:#x}  (not mapped)")
            continue
        lo, hi, off, dso = segs[i]
        rel = pc - lo + off
        # file offset -> virtual address of the DSO: the first mapping's base is offset 0
        base = min(s[0] - s[2] for s in segs if s[3] == dso)
        vaddr = pc - base
        sym = ""
        if os.path.exists(dso):
            if dso not in cache:
                cache[dso] = symbols(dso)
            syms = cache[dso]
            j = bisect.bisect_right([s[0] for s in syms], vaddr) - 1
            if j >= 0:
                sym = f"{syms[j][1]}+{vaddr - syms[j][0]:#x}"
        print(f"{pc:#x}  {os.path.basename(dso)}  file+{rel:#x}  vaddr {vaddr:#x}  {sym}")


if __name__ == "__main__":
    main()

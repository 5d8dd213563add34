"""Resolve the PCs of a glog "*** Aborted at ..." / SIGSEGV stack (as printed under rocprofv3) to
library + offset + symbol, using the /proc/self/maps dump written by tools/latency_split.py
(OMR_MAPS_OUT). The GPU box runs this container's image, so the same library files resolve here.
    python tools/resolve_stack.py <stack log> <maps file>"""
import re
import subprocess
import sys

SYMBOLIZER = "/opt/rocm/lib/llvm/bin/llvm-symbolizer"


def load_maps(path):
    maps = []
    for line in open(path):
        parts = line.split()
        if len(parts) < 6 or not parts[5].startswith("/"):
            continue
        lo, hi = (int(x, 16) for x in parts[0].split("-"))
        maps.append((lo, hi, int(parts[2], 16), parts[5]))
    return maps


def resolve(pc, maps):
    for lo, hi, off, path in maps:
        if lo <= pc < hi:
            # file offset of the PC; for PIE / shared objects the symbolizer wants the address
            # relative to the first (offset 0) mapping of the file
            base = min(l for l, _, o, p in maps if p == path and o == 0) if any(
                p == path and o == 0 for _, _, o, p in maps) else lo - off
            return path, pc - base
    return None, None


def main():
    log, maps_path = sys.argv[1], sys.argv[2]
    maps = load_maps(maps_path)
    for line in open(log):
        m = re.search(r"@\s+0x([0-9a-f]+)", line) or re.search(r"^PC: @\s+0x([0-9a-f]+)", line)
        if not m:
            continue
        pc = int(m.group(1), 16)
        path, rel = resolve(pc, maps)
        if path is None:
            print(f"0x{pc:x} ?")
            continue
        sym = ""
        try:
            sym = subprocess.run([SYMBOLIZER, "--obj", path, f"0x{rel:x}"], capture_output=True, text=True,
                                 timeout=60).stdout.split("\n")[0]
        except (OSError, subprocess.SubprocessError):
            pass
        print(f"0x{pc:x} {path}+0x{rel:x} {sym}")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table of one HIP unit, from the compiler's
kernel-resource-usage remarks (no GPU needed).

  python tools/kres.py bling_amd/csrc/core/prof_0.hip [-DKNOB=1 ...]
"""
import re
import subprocess
import sys

FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-gpu-rdc",
         "-munsafe-fp-atomics", "-Rpass-analysis=kernel-resource-usage", "-c", "-o", "/dev/null"]


def short(name: str) -> str:
    try:
        d = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-cxxfilt", name], capture_output=True, text=True).stdout.strip()
    except OSError:
        d = name
    d = re.sub(r"bd::DevScene const\*, bd::WaveState, ", "", d)
    d = re.sub(r"\(.*\)$", "", d)
    return d.replace("bd::", "").replace("bcore::", "")


def main():
    src, extra = sys.argv[1], sys.argv[2:]
    out = subprocess.run(["/opt/rocm/bin/hipcc"] + FLAGS + extra + [src], capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (.*?): (.*?) \[-Rpass", line)
        if not m:
            continue
        key, val = m.group(1).strip(), m.group(2).strip()
        if "Function Name" in line:
            cur = {"name": short(line.split("Function Name: ")[1].split(" [")[0])}
            rows.append(cur)
        elif cur is not None:
            cur[key] = val
    for r in rows:
        print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('AGPRs', '0'):>3} agpr  scratch {r.get('ScratchSize [bytes/lane]', '?'):>4}  "
              f"occ {r.get('Occupancy [waves/SIMD]', '?'):>2}  lds {r.get('LDS Size [bytes/block]', '?'):>6}  {r['name']}")


if __name__ == "__main__":
    main()

"""Per-kernel register / spill / LDS table of one HIP source (hipcc -Rpass-analysis=kernel-resource-usage).

usage: python scripts/kres.py imagecompression_adversarial_amd/csrc/ica_conv_x6.hip [name-filter] [-Dflags...]
"""
import os
import re
import subprocess
import sys


def main():
    src = os.path.abspath(sys.argv[1])
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src,
                          "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[3:],
                         capture_output=True, text=True, cwd="/tmp").stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    for r in rows:
        if filt not in r["name"]:
            continue
        dm = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
        dm = dm.replace("(anonymous namespace)::", "")[:80]
        print(f"{dm:80s} V{r.get('VGPRs', '?'):>4} A{r.get('AGPRs', '?'):>4} S{r.get('SGPRs', '?'):>4} "
              f"Vsp{r.get('VGPRs Spill', '?'):>4} Ssp{r.get('SGPRs Spill', '?'):>4} "
              f"LDS{r.get('LDS Size [bytes/block]', '?'):>7} occ{r.get('Occupancy [waves/SIMD]', '?')}")


if __name__ == "__main__":
    main()

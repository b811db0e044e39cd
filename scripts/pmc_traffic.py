"""HBM traffic per launch of the bench's tagged conv launches, from rocprofv3 --pmc passes (a FETCH_SIZE pass and
a WRITE_SIZE pass, run separately: scripts/gpu_pmc.sh), stamped with what was measured.

Which dispatch is which tag comes from the bench itself: scripts/gpu_pmc.sh runs bench.py with ICA_LAUNCH_TABLE set,
and bench.py writes {tag: [[kernel, grid_threads], ...]} of its timed launches (hip_ops.LAUNCH_HOOK, filled from the
library's ica_last_launch: the demangled name and Grid_Size rocprofv3 prints for the same dispatch).  A tag whose
launches all ran one (kernel, grid) is matched to the PMC rows of exactly that kernel and grid.

Correction (MI355X_MICROARCH.md, "HBM [CDNA4]"): on gfx950 FETCH_SIZE reports half the bytes of wide coalesced
streaming reads, so bytes_read = 2 * FETCH_SIZE (KB); WRITE_SIZE is exact for 16-B/lane stores.  The fp32 / x6
kernels load and store 16 B per lane (nChw4c float4), so both corrections apply as stated; the bf16 kernels' 8-B
quads make their corrected read figure an upper bound.

    python scripts/pmc_traffic.py <pmc dir> <launch table json> [label] > profiles/pmc_traffic_<cfg>.json

Output {tag: {"bytes", "read_bytes", "write_bytes", "kernel", "grid", "src"}}; "src" = hip_ops.source_hash() of the
tree that was measured.  bench.py reports an entry only when kernel, grid and src all match the launch it timed.
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def source_hash():
    # hip_ops.source_hash without importing torch / the library (same definition)
    import hashlib
    h = hashlib.sha256()
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "imagecompression_adversarial_amd", "csrc")
    for f in sorted(glob.glob(os.path.join(d, "*.hip")) + glob.glob(os.path.join(d, "*.h"))):
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def main():
    root, table = sys.argv[1], sys.argv[2]
    label = sys.argv[3] if len(sys.argv) > 3 else ""
    launches = json.load(open(table))
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{root}/p*/*_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            vals[(r["Kernel_Name"], int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))

    def med(v):
        v = sorted(v)
        return v[len(v) // 2]

    src = source_hash()
    out, skipped = {}, {}
    for tag, kl in sorted(launches.items()):
        kl = {tuple(k) for k in kl if k}
        if len(kl) != 1:
            skipped[tag] = f"{len(kl)} distinct (kernel, grid) pairs in the timed launches"
            continue
        name, grid = next(iter(kl))
        cs = vals.get((name, grid))
        if not cs or "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            skipped[tag] = "no FETCH_SIZE / WRITE_SIZE rows for that kernel and grid"
            continue
        rd = 2.0 * med(cs["FETCH_SIZE"]) * 1024
        wr = med(cs["WRITE_SIZE"]) * 1024
        out[tag] = {"bytes": round(rd + wr), "read_bytes": round(rd), "write_bytes": round(wr), "kernel": name,
                    "grid": grid, "src": src}
    json.dump({**out, "_skipped": skipped,
               "_note": "bytes per launch = 2*FETCH_SIZE + WRITE_SIZE (KB*1024), gfx950 correction per "
                        f"MI355X_MICROARCH.md HBM section; {label}"}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()

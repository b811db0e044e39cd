"""Summarise rocprofv3 --pmc CSVs per kernel (mean per dispatch) from gpurun_out/pmc/p*/."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
per = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
grid = {}
for f in sorted(glob.glob(f"{root}/p*/*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        key = (k, r["Grid_Size"])
        per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        dur[key].append(d)
        grid[key] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["LDS_Block_Size"])
rows = []
for key, cs in per.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    t = sorted(dur[key])[len(dur[key]) // 2]
    rows.append((t * sum(1 for _ in [0]), key, m, t))
rows.sort(key=lambda x: -x[3])
for _, (k, g), m, t in rows[:16]:
    name = k.split("(")[0][:44]
    out = [f"{name:44s} grid={g:>8} t={t*1e3:7.3f}ms vgpr/agpr/lds={grid[(k,g)]}"]
    if "GRBM_GUI_ACTIVE" in m:
        out.append(f"clk={m['GRBM_GUI_ACTIVE'] / 8 / t / 1e9:.2f}GHz")
    if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"] > 0:
        w = m["SQ_WAVE_CYCLES"]
        out.append(f"wait={m.get('SQ_WAIT_ANY', 0)/w:.2f} waitinst={m.get('SQ_WAIT_INST_ANY', 0)/w:.2f} "
                   f"active={m.get('SQ_ACTIVE_INST_ANY', 0)/w:.2f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
        # MFMA busy cycles summed over SIMDs; per-SIMD utilisation vs elapsed cycles
        out.append(f"mfma_busy={m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * 1024):.2f}")
    if "FETCH_SIZE" in m:
        out.append(f"fetchKB(x2)={2 * m['FETCH_SIZE']:.0f}")
    if "WRITE_SIZE" in m:
        out.append(f"writeKB={m['WRITE_SIZE']:.0f}")
    for c in ("SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
              "SQ_INSTS_SALU", "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS", "TCP_TOTAL_CACHE_ACCESSES_sum",
              "TCP_TCC_READ_REQ_sum", "TCC_HIT_sum", "TCC_MISS_sum"):
        if c in m:
            out.append(f"{c[8:]}={m[c]:.3g}")
    print(" | ".join(out))

"""HBM traffic per launch of the bench's tagged g_a / g_s kernels, from rocprofv3 --pmc passes
(FETCH_SIZE pass and WRITE_SIZE pass, run separately: scripts/gpu_pmc.sh).

Correction (MI355X_MICROARCH.md, "HBM [CDNA4]"): on gfx950 FETCH_SIZE reports half the bytes of wide
coalesced streaming reads, so bytes_read = 2 * FETCH_SIZE (KB); WRITE_SIZE is exact for 16-B/lane stores.
Our loads/stores are 16 B per lane (nChw4c float4), so both corrections apply as stated.

Kernels are identified by (name prefix, Grid_Size); the grids follow the launchers in ica_conv.hip.
    python scripts/pmc_traffic.py gpurun_out/pmc [B H W prec] > profiles/pmc_traffic.json
(default: 32 x 512x768 fp32; config 2 x6 = 32 512 768 x6; config 5 = 8 2048 2048 bf16; config 3 = 32 512 768
cheng_x6).  Output {tag: bytes/launch}.
"""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
B, H, W = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (32, 512, 768)
PREC = sys.argv[5] if len(sys.argv) > 5 else "fp32"
BF = "true" if PREC == "bf16" else "false"
TH = {32: 4, 16: 8}


def tw(Wout):
    return 32 if Wout >= 32 and Wout % 32 == 0 else 16


def down(cc, epi, Hout, Wout, Cout, it):
    t = tw(Wout)
    th = (256 if (PREC == "bf16" and cc == 16) else 128) // t   # bf16 16-channel chunks: 2 pixel tiles per wave
    grid = -(-Wout // t) * -(-Hout // th) * B * 256 * -(-Cout // (it * 32))
    return f"void conv_down_kernel<5, 2, {it}, {cc}, {t}, {epi}, 0, {BF}>", grid


def up(epi, Hin, Win, Cout, it):
    th = 8 if PREC == "bf16" else 4   # bf16: two 32-pixel tiles per class per wave
    return f"void conv_up_kernel<5, {it}, {epi}, 0, {BF}>", -(-Win // 16) * -(-Hin // th) * B * 256 * -(-Cout // (it * 32))


def up3(Hin, Win):
    return f"void conv_up3_kernel<{BF}>", -(-Win // 32) * -(-Hin // 5) * B * 256   # 5x32 input tiles


N, M = 128, 192
h = [(H >> k, W >> k) for k in range(5)]   # resolution of level k
TAGS = {   # epilogue ids: 0 BIAS, 2 GDN, 3 IGDN, 4 GDN_BWD, 5 IGDN_BWD
    "g_a.0.fwd": down(4, 2, *h[1], N, 4), "g_a.2.fwd": down(16, 2, *h[2], N, 4),
    "g_a.4.fwd": down(16, 2, *h[3], N, 4), "g_a.6.fwd": down(16, 0, *h[4], M, 3),
    "g_s.0.fwd": up(3, *h[4], N, 4), "g_s.2.fwd": up(3, *h[3], N, 4), "g_s.4.fwd": up(3, *h[2], N, 4),
    "g_s.6.fwd": up3(*h[1]),    # shares its name and grid with g_a.0.dgrad
    "g_s.6.dgrad": down(4, 5, *h[1], N, 4), "g_s.4.dgrad": down(16, 5, *h[2], N, 4),
    "g_s.2.dgrad": down(16, 5, *h[3], N, 4), "g_s.0.dgrad": down(16, 0, *h[4], M, 3),
    "g_a.6.dgrad": up(4, *h[4], N, 4), "g_a.4.dgrad": up(4, *h[3], N, 4), "g_a.2.dgrad": up(4, *h[2], N, 4),
    "g_a.0.dgrad": up3(*h[1]),
}

if PREC == "x6":   # ica_conv_x6.hip launchers (and the x6 conv_up3); names carry the PT template argument
    NS = "void (anonymous namespace)::"

    def down_x6(epi, Hout, Wout, Cout, it):
        ncb = -(-Cout // (it * 32))
        b2 = -(-Wout // 32) * -(-Hout // 8) * B * ncb
        pt = 2 if b2 >= 256 else 1
        return f"{NS}conv_down_x6_kernel<{it}, {epi}, {pt}>", -(-Wout // 32) * -(-Hout // (4 * pt)) * B * 256 * ncb

    def rgb_x6(epi, Hout, Wout, Cout):
        tiles = -(-Wout // 32) * -(-Hout // 4) * B
        if epi in (4, 5):   # persistent GDN-backward form: one block per CU, contiguous tile runs
            per = -(-tiles // min(tiles, 256))
            return f"{NS}conv_rgb_bwd_x6_kernel<4, {epi}>", -(-tiles // per) * 256
        return f"{NS}conv_rgb_x6_kernel<4, {epi}>", tiles * 256 * -(-Cout // 128)

    def up_x6(epi, Hin, Win, Cin, Cout):
        cg = 128 if Cin <= 128 else 64
        ncb = -(-Cout // 128)
        fill = lambda n: n / (-(-n // 256) * 256)   # noqa: E731  (launch_up_x6's round fill)
        b2 = -(-Win // 16) * -(-Hin // 8) * B * ncb
        b1 = -(-Win // 16) * -(-Hin // 4) * B * ncb
        pt = 1 if fill(b1) > fill(b2) + 0.15 else 2
        return f"{NS}conv_up_x6_kernel<4, {epi}, {cg}, {pt}>", (b1 if pt == 1 else b2) * 256

    def up3_x6(Hin, Win):
        ct = 3   # Cin = 128: 10 x 30 input tiles, persistent
        tiles = -(-Win // 30) * -(-Hin // (4 * ct - 2)) * B
        per = -(-tiles // min(tiles, 256))
        return "void conv_up3_x6p_kernel<8, 3>", -(-tiles // per) * 256

    TAGS = {
        "g_a.0.fwd": rgb_x6(2, *h[1], N), "g_a.2.fwd": down_x6(2, *h[2], N, 4),
        "g_a.4.fwd": down_x6(2, *h[3], N, 4), "g_a.6.fwd": down_x6(0, *h[4], M, 3),
        "g_s.0.fwd": up_x6(3, *h[4], M, N), "g_s.2.fwd": up_x6(3, *h[3], N, N), "g_s.4.fwd": up_x6(3, *h[2], N, N),
        "g_s.6.fwd": up3_x6(*h[1]),    # shares its name and grid with g_a.0.dgrad
        "g_s.6.dgrad": rgb_x6(5, *h[1], N), "g_s.4.dgrad": down_x6(5, *h[2], N, 4),
        "g_s.2.dgrad": down_x6(5, *h[3], N, 4), "g_s.0.dgrad": down_x6(0, *h[4], M, 3),
        "g_a.6.dgrad": up_x6(4, *h[4], M, N), "g_a.4.dgrad": up_x6(4, *h[3], N, N), "g_a.2.dgrad": up_x6(4, *h[2], N, N),
        "g_a.0.dgrad": up3_x6(*h[1]),
    }

if PREC == "cheng_x6":   # cheng2020 q6 on x6 operands (config 3): the full-resolution k3 s1 launches with a
    # (kernel, grid) of their own (conv_down_kernel X6O: 32 x 4 output pixels per block, IT = 6, Cout = 192)
    def k3x6(epi, fx, Hout, Wout):
        return (f"void conv_down_kernel<3, 1, 6, 16, 32, {epi}, {fx}, false, true>",
                -(-Wout // 32) * -(-Hout // 4) * B * 256)

    TAGS = {"g_s.6.conv1.dgrad": k3x6(5, 1, *h[1]), "g_a.1.conv1.dgrad": k3x6(4, 1, *h[1]),
            "g_a.0.conv2.fwd": k3x6(2, 1, *h[1]), "g_s.5.conv.fwd": k3x6(3, 1, *h[1])}

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/p*/*_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        vals[(r["Kernel_Name"], int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))


def med(v):
    v = sorted(v)
    return v[len(v) // 2]


out, detail = {}, {}
for tag, (prefix, grid) in TAGS.items():
    hits = [cs for (k, g), cs in vals.items() if k.startswith(prefix) and g == grid]
    if not hits or "FETCH_SIZE" not in hits[0] or "WRITE_SIZE" not in hits[0]:
        continue
    cs = hits[0]
    rd = 2.0 * med(cs["FETCH_SIZE"]) * 1024
    wr = med(cs["WRITE_SIZE"]) * 1024
    out[tag] = rd + wr
    detail[tag] = {"read_bytes": rd, "write_bytes": wr}
json.dump({**{k: round(v) for k, v in out.items()}, "_detail": detail,
           "_note": f"bytes per launch = 2*FETCH_SIZE + WRITE_SIZE (KB*1024), gfx950 correction per "
                    f"MI355X_MICROARCH.md HBM section; {'cheng2020 q6' if PREC == 'cheng_x6' else 'hyper q3'}, "
                    f"{B} x {H}x{W}, {PREC} conv operands"},
          sys.stdout, indent=1)
print()

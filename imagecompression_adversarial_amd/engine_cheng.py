"""cheng2020-anchor on the HIP conv engine (CompressAI Cheng2020Anchor built at
anchors/model.py:76-77, composed at anchors/model.py:97-106).

Every layer is one ``ica_conv_ex`` launch with its elementwise work fused into the epilogue or the
LDS fill (N = 192 channels run as one 6-tile MFMA wave so GDN's channel GEMM stays in registers):

  forward                                   epilogue / fill
  RBS  conv3x3 s2 -> LReLU                  EPI_LRELU                        (saves a1)
       conv1x1 s2 skip                      EPI_BIAS                         -> r
       conv3x3 -> GDN, + r                  EPI_GDN, res=r                   (saves y_gdn, s)
  RB   conv3x3 -> LReLU                     EPI_LRELU                        (saves a1)
       conv3x3 -> LReLU, + x                EPI_LRELU, res=x                 (saves a2)
  RBU  subpel conv3x3 -> PixelShuffle -> LReLU   EPI_LRELU, ps               (saves a1)
       subpel conv3x3 (upsample) -> PixelShuffle EPI_BIAS, ps                -> r
       conv3x3 -> IGDN, + r                 EPI_IGDN, res=r                  (saves y_igdn, s)
  backward (input gradients only)
  RB   g*lrelu'(a2) -> conv3x3^T -> *lrelu'(a1)     fill_mode 1 + EPI_LRELU_BWD
       conv3x3^T + g [-> GDN/IGDN bwd of the block before, saving the summed g]   res (+ EPI_*GDN_BWD)
  RBS  conv3x3^T -> *lrelu'(a1); skip^T (1x1 s2 transposed); conv3x3 s2^T + skip^T   conv_up KS=3/1
  RBU  conv3x3^T -> *lrelu'(a1); unshuffle -> subpel^T; unshuffle -> upsample^T + ...  fill_mode 2

Tensors are nChw4c (hip_ops).  Subpel weights / biases are re-ordered host-side into the rho row order
the PixelShuffle store and the PixelUnshuffle fill expect (rho = 16*c4 + 4*q + e <-> channel 4*(4c4+e)+q).
"""
from __future__ import annotations

import torch

from . import hip_ops as K


def _k(prefix, name):
    return f"{prefix}.{name}" if prefix else name


def _it(C):
    """32-channel row tiles per wave: 6 for N = 192 (q4-6), 4 for N = 128 (q1-3; explicit, so the x6 / bf16 packs
    below are built for it too), 1 for the 3- and 16-row layers, else the library default."""
    return 6 if C == 192 else (4 if C == 128 else (1 if C <= 32 else 0))


def rho_perm(C: int, device) -> torch.Tensor:
    """Index map rho -> PixelShuffle(2) input channel (4C rows; -1 marks padding rows when C % 4)."""
    C4 = (C + 3) // 4
    idx = torch.full((16 * C4,), -1, dtype=torch.long)
    for c4 in range(C4):
        for q in range(4):
            for e in range(4):
                c = 4 * c4 + e
                if c < C:
                    idx[16 * c4 + 4 * q + e] = 4 * c + q
    return idx.to(device)


def _rho_weight(w, b, C):
    """Subpel conv weight [4C][Cin][3][3] / bias [4C] -> rho order [16*ceil(C/4)][Cin][3][3] (zero padding)."""
    idx = rho_perm(C, w.device)
    keep = (idx >= 0).to(w.dtype)
    safe = idx.clamp_min(0)
    wr = w.detach()[safe] * keep.view(-1, 1, 1, 1)
    br = b.detach()[safe] * keep
    return wr.contiguous(), br.contiguous()


X6_IT = (4, 6)   # row tiles of the x6 k3 s1 conv_down instantiations (ica_conv.hip pick_down_x6o)
X6_IT_PS = (1, 4, 6)   # ... and of the subpel forwards (IT = 1: g_s.7's 16 rho rows, bias + PixelShuffle only)


class Conv3:
    """One Conv2d(k in {1,3,5}, stride s, pad k//2) layer, packed for its forward and its input gradient."""

    def __init__(self, w, b, stride=1, fwd_only=False, mask=None, x6=False, b1=False):
        """b1 (with x6): the X6O conv_down launches (k3 s1 forward / input gradient, k3 s2 forward) run bf16
        operands over fp32 activations (hip_ops.PREC_B1: the x6 pack's hi plane); the stride-2 input gradients keep
        x6 (cheng2020 --precision bf16)."""
        w = w.detach()
        self.p6 = K.PREC_B1 if b1 else K.PREC_X6
        if mask is not None:
            w = (w * mask.to(w.device)).contiguous()
        self.Cout, self.Cin, self.KS = w.shape[0], w.shape[1], w.shape[-1]
        self.S = stride
        KK = self.KS * self.KS
        self.it = _it(self.Cout)
        cc = 4 if self.Cin <= 4 else 16
        self.fwd = K.pack_conv(w, self.Cout, self.Cin, self.KS, self.Cin * KK, KK, K.ORDER_DOWN, cc, it=self.it)
        self.bias = None if b is None else b.detach().contiguous()
        self.bwd = None
        self.it_b = _it(self.Cin)
        if not fwd_only:
            if stride == 1:   # dgrad = conv with the taps reversed, channels swapped
                self.bwd = K.pack_conv(w, self.Cin, self.Cout, self.KS, KK, self.Cin * KK, K.ORDER_DOWN, 16,
                                       flip=True, it=self.it_b)
            else:             # dgrad = stride-2 transposed conv (conv_up, KS in {3, 1})
                self.bwd = K.pack_conv(w, self.Cin, self.Cout, self.KS, KK, self.Cin * KK, K.ORDER_UP, 16,
                                       it=self.it_b)
        # x6 operands (fp32-accurate bf16x6) for the k3 s1 layers: three-plane packs of the same fragment orders
        # (the input gradient's taps reversed by flipping the weight); launches that write t keep the fp32 packs
        self.fwd6 = self.bwd6 = None
        if (x6 and stride == 2 and self.KS in (1, 3) and not fwd_only and self.Cin in (128, 192)
                and self.it_b in X6_IT):
            # the k3 s2 input gradient (x6 conv_up, ica_conv_x6.hip pick_up3s2_x6) and the 1x1 s2 skips' (one tap in
            # output class (0, 0)): conv_up fragment order
            self.bwd6 = K.pack_conv_x6(w, self.Cin, self.Cout, self.KS, KK, self.Cin * KK, K.ORDER_UP, self.it_b)
        if x6 and stride == 2 and self.KS == 3 and self.Cin >= 16 and mask is None and self.it in X6_IT:
            # the k3 s2 forward (cheng2020 g_a.2 / g_a.4 conv1, leaky ReLU; ica_conv.hip pick_down_x6o_s2)
            self.fwd6 = K.pack_conv_x6(w, self.Cout, self.Cin, 3, self.Cin * KK, KK, K.ORDER_DOWN, self.it)
        if x6 and stride == 1 and self.KS == 3 and self.Cin >= 16 and mask is None and self.it in X6_IT:
            self.fwd6 = K.pack_conv_x6(w, self.Cout, self.Cin, 3, self.Cin * KK, KK, K.ORDER_DOWN, self.it)
            if not fwd_only and self.Cout >= 16 and self.it_b in X6_IT:
                self.bwd6 = K.pack_conv_x6(w.flip(-1, -2).contiguous(), self.Cin, self.Cout, 3, KK, self.Cin * KK,
                                           K.ORDER_DOWN, self.it_b)

    def forward(self, x4, epi=K.EPI_BIAS, **kw):
        if self.fwd6 is not None and _x6_ok(kw):
            return K.conv_ex(x4, self.Cin, self.fwd6, self.bias, self.Cout, self.KS, self.S, 0, epi, self.it,
                             prec=self.p6, **kw)
        return K.conv_ex(x4, self.Cin, self.fwd, self.bias, self.Cout, self.KS, self.S, 0, epi, self.it, **kw)

    def dgrad(self, g4, epi=K.EPI_BIAS, **kw):
        if self.S == 1:
            if self.bwd6 is not None and _x6_ok(kw):
                return K.conv_ex(g4, self.Cout, self.bwd6, None, self.Cin, self.KS, 1, 0, epi, self.it_b,
                                 prec=self.p6, **kw)
            return K.conv_ex(g4, self.Cout, self.bwd, None, self.Cin, self.KS, 1, 0, epi, self.it_b, **kw)
        if self.bwd6 is not None and epi == K.EPI_BIAS and _x6_ok(kw):
            return K.conv_ex(g4, self.Cout, self.bwd6, None, self.Cin, self.KS, 2, 1, epi, self.it_b,
                             prec=K.PREC_X6, **kw)
        return K.conv_ex(g4, self.Cout, self.bwd, None, self.Cin, self.KS, 2, 1, epi, self.it_b, **kw)


def _x6_ok(kw):
    """An x6 k3 s1 launch: any fill (plain, leaky-ReLU mask, PixelUnshuffle), no t output (ica_conv.hip
    pick_down_x6o)."""
    return kw.get("save_t") is None


class Subpel:
    """subpel_conv3x3(Cin, C, 2) = Conv2d(Cin, 4C, 3, p=1) + PixelShuffle(2), rho-ordered rows."""

    def __init__(self, w, b, fwd_only=False, x6=False, b1=False):
        self.p6 = K.PREC_B1 if b1 else K.PREC_X6   # as Conv3
        self.C = w.shape[0] // 4
        self.Cin = w.shape[1]
        wr, self.bias = _rho_weight(w, b, self.C)
        self.R = wr.shape[0]          # rho rows = 16 * ceil(C / 4)
        self.it = 6 if self.R == 768 else (4 if self.R % 128 == 0 else _it(self.R))   # N = 192 / 128 / g_s.7
        self.fwd = K.pack_conv(wr, self.R, self.Cin, 3, self.Cin * 9, 9, K.ORDER_DOWN, 16, it=self.it)
        # x6 forward (PixelShuffle store) and input gradient (PixelUnshuffle fill, the flipped weight)
        self.fwd6 = (K.pack_conv_x6(wr, self.R, self.Cin, 3, self.Cin * 9, 9, K.ORDER_DOWN, self.it)
                     if x6 and self.Cin >= 16 and self.it in X6_IT_PS else None)
        self.it_b = _it(self.Cin)
        self.bwd = None if fwd_only else K.pack_conv(wr, self.Cin, self.R, 3, 9, self.Cin * 9, K.ORDER_DOWN, 16,
                                                     flip=True, it=self.it_b)
        self.bwd6 = (K.pack_conv_x6(wr.flip(-1, -2).contiguous(), self.Cin, self.R, 3, 9, self.Cin * 9,
                                    K.ORDER_DOWN, self.it_b)
                     if x6 and not fwd_only and self.R >= 16 and self.it_b in X6_IT else None)

    def forward(self, x4, epi=K.EPI_BIAS, **kw):
        # x6 at IT = 1 (g_s.7's 16 rho rows) is built for the bias epilogue only (ica_conv.hip pick_down_x6o)
        if self.fwd6 is not None and _x6_ok(kw) and (self.it != 1 or epi == K.EPI_BIAS):
            return K.conv_ex(x4, self.Cin, self.fwd6, self.bias, self.R, 3, 1, 0, epi, self.it, ps=True,
                             alg_rows=4 * self.C, prec=self.p6, **kw)
        return K.conv_ex(x4, self.Cin, self.fwd, self.bias, self.R, 3, 1, 0, epi, self.it, ps=True,
                         alg_rows=4 * self.C, **kw)

    def dgrad(self, g4, **kw):
        """g4: gradient of the shuffled output [N, C/4, 2H, 2W, 4] -> gradient of the input [N, Cin, H, W]."""
        if self.bwd6 is not None and _x6_ok(kw):
            return K.conv_ex(g4, self.R, self.bwd6, None, self.Cin, 3, 1, 0, K.EPI_BIAS, self.it_b,
                             fill_mode=K.FILL_UNSHUFFLE, alg_rows=4 * self.C, prec=self.p6, **kw)
        return K.conv_ex(g4, self.R, self.bwd, None, self.Cin, 3, 1, 0, K.EPI_BIAS, self.it_b,
                         fill_mode=K.FILL_UNSHUFFLE, alg_rows=4 * self.C, **kw)


def _gdn(sd, pre):
    return K.PackedGDN(sd[f"{pre}.beta"], sd[f"{pre}.gamma"])


class ChengAnalysis:
    """g_a = RBS(3,N) RB RBS RB RBS RB conv3x3 s2."""

    def __init__(self, sd, prefix="g_a", tag="g_a", x6=False, b1=False):
        self.tag = tag
        self.N = sd[_k(prefix, "6.weight")].shape[0]
        self.M = self.N
        self.blocks = []
        for i in range(6):
            pre = _k(prefix, str(i))
            if i % 2 == 0:
                self.blocks.append(("rbs", Conv3(sd[f"{pre}.conv1.weight"], sd[f"{pre}.conv1.bias"], 2, x6=x6, b1=b1),
                                    Conv3(sd[f"{pre}.conv2.weight"], sd[f"{pre}.conv2.bias"], 1, x6=x6, b1=b1),
                                    Conv3(sd[f"{pre}.skip.weight"], sd[f"{pre}.skip.bias"], 2, x6=x6, b1=b1),
                                    _gdn(sd, f"{pre}.gdn")))
            else:
                self.blocks.append(("rb", Conv3(sd[f"{pre}.conv1.weight"], sd[f"{pre}.conv1.bias"], 1, x6=x6, b1=b1),
                                    Conv3(sd[f"{pre}.conv2.weight"], sd[f"{pre}.conv2.bias"], 1, x6=x6, b1=b1)))
        self.last = Conv3(sd[_k(prefix, "6.weight")], sd[_k(prefix, "6.bias")], 2)
        # x6: the image-side block's two input gradients (conv1 k3 s2 and skip k1 s2 into 3 channels) as one fused
        # Z-gather launch (ica_conv_up3k3_x6) instead of two 32-row fp32 conv_up tiles computing 3 rows each
        w1, wsk = sd[_k(prefix, "0.conv1.weight")], sd[_k(prefix, "0.skip.weight")]
        self.rgb6 = (K.pack_up3k3_x6(w1, wsk) if x6 and w1.shape[1] == 3 and w1.shape[0] % 16 == 0
                     and tuple(wsk.shape[1:]) == (3, 1, 1) else None)

    def forward(self, x4, save=False, inputs=None):
        """inputs: an optional list that receives every block's input and the last conv's (the weight gradients of
        the fine-tune, train_cheng)."""
        h, saved = x4, []
        for i, blk in enumerate(self.blocks):
            t = f"{self.tag}.{i}"
            if inputs is not None:
                inputs.append(h)
            if blk[0] == "rbs":
                _, c1, c2, sk, gd = blk
                a1 = c1.forward(h, K.EPI_LRELU, tag=f"{t}.conv1.fwd")
                r = sk.forward(h, K.EPI_BIAS, tag=f"{t}.skip.fwd")
                yg = torch.empty_like(r) if save else None
                s = torch.empty_like(r) if save else None
                h = c2.forward(a1, K.EPI_GDN, gdn=gd, res=r, save_x=yg, save_s=s, tag=f"{t}.conv2.fwd")
                del r
                if save and i == 0:
                    a1._ica_in_hw = (x4.shape[2], x4.shape[3])   # the image size, for the fused input gradient
                saved.append((a1, yg, s) if save else None)
            else:
                _, c1, c2 = blk
                a1 = c1.forward(h, K.EPI_LRELU, tag=f"{t}.conv1.fwd")
                a2 = torch.empty_like(a1) if save else None
                h = c2.forward(a1, K.EPI_LRELU, res=h, save_x=a2, tag=f"{t}.conv2.fwd")
                saved.append((a1, a2) if save else None)
        if inputs is not None:
            inputs.append(h)
        y = self.last.forward(h, K.EPI_BIAS, tag=f"{self.tag}.6.fwd")
        return y, saved

    def backward(self, gy4, saved):
        g = self.last.dgrad(gy4, tag=f"{self.tag}.6.dgrad")
        g_sum = None
        for i in range(5, -1, -1):
            blk, sv, t = self.blocks[i], saved[i], f"{self.tag}.{i}"
            if blk[0] == "rb":
                _, c1, c2 = blk
                a1, a2 = sv
                gc1 = c2.dgrad(g, K.EPI_LRELU_BWD, fill_mode=K.FILL_LRELU_MASK, mask=a2, saved=(a1, None),
                               tag=f"{t}.conv2.dgrad")
                # the block before is an RBS: fuse its GDN backward (+ keep the summed gradient for its skip)
                _, _, _, _, gd = self.blocks[i - 1]
                g_sum = torch.empty_like(g)
                g = c1.dgrad(gc1, K.EPI_GDN_BWD, gdn=gd, res=g, save_x=g_sum, saved=saved[i - 1][1:],
                             tag=f"{t}.conv1.dgrad")
            else:
                _, c1, c2, sk, gd = blk
                a1 = sv[0]
                gc1 = c2.dgrad(g, K.EPI_LRELU_BWD, saved=(a1, None), tag=f"{t}.conv2.dgrad")
                hw = getattr(a1, "_ica_in_hw", None)
                if (i == 0 and self.rgb6 is not None and hw is not None and (hw[0] + 1) // 2 == gc1.shape[2]
                        and (hw[1] + 1) // 2 == gc1.shape[3]):
                    g = K.conv_up3k3_x6(gc1, g_sum, self.rgb6, hw[0], hw[1], tag=f"{t}.conv1+skip.dgrad")
                    continue
                r = sk.dgrad(g_sum, tag=f"{t}.skip.dgrad")
                g = c1.dgrad(gc1, K.EPI_BIAS, res=r, tag=f"{t}.conv1.dgrad")
                del r
        return g


class ChengSynthesis:
    """g_s = RB RBU RB RBU RB RBU RB subpel_conv3x3(N, 3, 2)."""

    def __init__(self, sd, prefix="g_s", tag="g_s", x6=False, b1=False):
        self.tag = tag
        self.N = sd[_k(prefix, "0.conv1.weight")].shape[0]
        self.M = self.N
        self.blocks = []
        for i in range(7):
            pre = _k(prefix, str(i))
            if i % 2 == 0:
                self.blocks.append(("rb", Conv3(sd[f"{pre}.conv1.weight"], sd[f"{pre}.conv1.bias"], 1, x6=x6, b1=b1),
                                    Conv3(sd[f"{pre}.conv2.weight"], sd[f"{pre}.conv2.bias"], 1, x6=x6, b1=b1)))
            else:
                self.blocks.append(("rbu", Subpel(sd[f"{pre}.subpel_conv.0.weight"], sd[f"{pre}.subpel_conv.0.bias"],
                                                  x6=x6, b1=b1),
                                    Conv3(sd[f"{pre}.conv.weight"], sd[f"{pre}.conv.bias"], 1, x6=x6, b1=b1),
                                    Subpel(sd[f"{pre}.upsample.0.weight"], sd[f"{pre}.upsample.0.bias"], x6=x6, b1=b1),
                                    _gdn(sd, f"{pre}.igdn")))
        self.last = Subpel(sd[_k(prefix, "7.0.weight")], sd[_k(prefix, "7.0.bias")], x6=x6, b1=b1)

    def forward(self, y4, save=False, inputs=None):
        """inputs: as ChengAnalysis.forward."""
        h, saved = y4, []
        for i, blk in enumerate(self.blocks):
            t = f"{self.tag}.{i}"
            if inputs is not None:
                inputs.append(h)
            if blk[0] == "rb":
                _, c1, c2 = blk
                a1 = c1.forward(h, K.EPI_LRELU, tag=f"{t}.conv1.fwd")
                a2 = torch.empty_like(a1) if save else None
                h = c2.forward(a1, K.EPI_LRELU, res=h, save_x=a2, tag=f"{t}.conv2.fwd")
                saved.append((a1, a2) if save else None)
            else:
                _, sp, cv, up, gd = blk
                a1 = sp.forward(h, K.EPI_LRELU, tag=f"{t}.subpel.fwd")
                r = up.forward(h, K.EPI_BIAS, tag=f"{t}.upsample.fwd")
                yg = torch.empty_like(r) if save else None
                s = torch.empty_like(r) if save else None
                h = cv.forward(a1, K.EPI_IGDN, gdn=gd, res=r, save_x=yg, save_s=s, tag=f"{t}.conv.fwd")
                del r
                saved.append((a1, yg, s) if save else None)
        if inputs is not None:
            inputs.append(h)
        xh = self.last.forward(h, K.EPI_BIAS, tag=f"{self.tag}.7.fwd")
        return xh, saved

    def backward(self, gx4, saved):
        g = self.last.dgrad(gx4, tag=f"{self.tag}.7.dgrad")
        g_sum = None
        for i in range(6, -1, -1):
            blk, sv, t = self.blocks[i], saved[i], f"{self.tag}.{i}"
            if blk[0] == "rb":
                _, c1, c2 = blk
                a1, a2 = sv
                gc1 = c2.dgrad(g, K.EPI_LRELU_BWD, fill_mode=K.FILL_LRELU_MASK, mask=a2, saved=(a1, None),
                               tag=f"{t}.conv2.dgrad")
                if i == 0:
                    g = c1.dgrad(gc1, K.EPI_BIAS, res=g, tag=f"{t}.conv1.dgrad")
                else:
                    _, _, _, _, gd = self.blocks[i - 1]
                    g_sum = torch.empty_like(g)
                    g = c1.dgrad(gc1, K.EPI_IGDN_BWD, gdn=gd, res=g, save_x=g_sum, saved=saved[i - 1][1:],
                                 tag=f"{t}.conv1.dgrad")
            else:
                _, sp, cv, up, gd = blk
                a1 = sv[0]
                ga1 = cv.dgrad(g, K.EPI_LRELU_BWD, saved=(a1, None), tag=f"{t}.conv.dgrad")
                part = sp.dgrad(ga1, tag=f"{t}.subpel.dgrad")
                g = up.dgrad(g_sum, res=part, tag=f"{t}.upsample.dgrad")
                del part
        return g


class ChengHA:
    """h_a = conv3x3-LReLU-conv3x3-LReLU-conv3x3 s2-LReLU-conv3x3-LReLU-conv3x3 s2 (forward only)."""

    def __init__(self, sd, prefix="h_a"):
        self.convs = [Conv3(sd[_k(prefix, f"{i}.weight")], sd[_k(prefix, f"{i}.bias")], 2 if i in (4, 8) else 1,
                            fwd_only=True) for i in (0, 2, 4, 6, 8)]
        self.out_channels = self.convs[-1].Cout

    def forward(self, y4):
        z = y4
        for j, c in enumerate(self.convs):
            z = c.forward(z, K.EPI_LRELU if j < 4 else K.EPI_BIAS)
        return z


class ChengHS:
    """h_s = conv3x3-LReLU-subpel-LReLU-conv3x3(N,3N/2)-LReLU-subpel-LReLU-conv3x3(3N/2,2N) (forward only)."""

    def __init__(self, sd, prefix="h_s"):
        self.c0 = Conv3(sd[_k(prefix, "0.weight")], sd[_k(prefix, "0.bias")], 1, fwd_only=True)
        self.s2 = Subpel(sd[_k(prefix, "2.0.weight")], sd[_k(prefix, "2.0.bias")], fwd_only=True)
        self.c4 = Conv3(sd[_k(prefix, "4.weight")], sd[_k(prefix, "4.bias")], 1, fwd_only=True)
        self.s6 = Subpel(sd[_k(prefix, "6.0.weight")], sd[_k(prefix, "6.0.bias")], fwd_only=True)
        self.c8 = Conv3(sd[_k(prefix, "8.weight")], sd[_k(prefix, "8.bias")], 1, fwd_only=True)
        self.out_channels = self.c8.Cout

    def forward(self, z4):
        s = self.c0.forward(z4, K.EPI_LRELU)
        s = self.s2.forward(s, K.EPI_LRELU)
        s = self.c4.forward(s, K.EPI_LRELU)
        s = self.s6.forward(s, K.EPI_LRELU)
        return self.c8.forward(s, K.EPI_BIAS)


def context_mask(k):
    """MaskedConv2d type 'A' (raster order: centre tap and everything after it zeroed)."""
    m = torch.ones(k, k)
    m[k // 2, k // 2:] = 0
    m[k // 2 + 1:] = 0
    return m


class ChengContext:
    """context_prediction = MaskedConv2d(N, 2N, 5, padding=1... 2) type A (forward only)."""

    def __init__(self, sd, prefix="context_prediction"):
        w = sd[_k(prefix, "weight")]
        self.conv = Conv3(w, sd[_k(prefix, "bias")], 1, fwd_only=True, mask=context_mask(w.shape[-1]))
        self.out_channels = self.conv.Cout

    def forward(self, y_hat4):
        return self.conv.forward(y_hat4, K.EPI_BIAS)


class ChengEntropyParameters:
    """entropy_parameters = conv1x1-LReLU-conv1x1-LReLU-conv1x1 (forward only)."""

    def __init__(self, sd, prefix="entropy_parameters"):
        self.convs = [Conv3(sd[_k(prefix, f"{i}.weight")], sd[_k(prefix, f"{i}.bias")], 1, fwd_only=True)
                      for i in (0, 2, 4)]
        self.out_channels = self.convs[-1].Cout

    def forward(self, t4):
        t = self.convs[0].forward(t4, K.EPI_LRELU)
        t = self.convs[1].forward(t, K.EPI_LRELU)
        return self.convs[2].forward(t, K.EPI_BIAS)


class ChengKernels:
    """CodecKernels-compatible executor for cheng2020-anchor (g_a/g_s fwd+dgrad, eval forward)."""

    model = "cheng2020"

    def __init__(self, sd: dict, precision: str = "fp32"):
        """precision 'x6': the k3 layers of g_a / g_s (the bulk of the work) on fp32-accurate bf16x6 operands
        (Conv3 / Subpel / rgb6 above list which launches); 'bf16': the same launches with the k3 conv_downs on bf16
        operands over fp32 activations (hip_ops.PREC_B1; the stride-2 input gradients stay x6); the rest fp32."""
        if sd["g_a.6.weight"].device.type != "cuda":
            raise RuntimeError("ChengKernels needs the state dict on the HIP device")
        if precision not in ("fp32", "x6", "bf16"):
            raise NotImplementedError(f"cheng2020 operands: fp32, x6 or bf16, not {precision!r}")
        x6, b1 = precision in ("x6", "bf16"), precision == "bf16"
        self.ga = ChengAnalysis(sd, x6=x6, b1=b1)
        self.gs = ChengSynthesis(sd, x6=x6, b1=b1)
        self.N = self.M = self.ga.N
        self.ha = ChengHA(sd)
        self.hs = ChengHS(sd)
        self.ctx = ChengContext(sd)
        self.ep = ChengEntropyParameters(sd)
        self.eb = K.PackedEB({n: sd[f"entropy_bottleneck.{n}"] for n in K.PackedEB.NAMES})

    def g_a(self, x4, save=False):
        return self.ga.forward(x4, save)

    def g_a_backward(self, gy4, saved):
        return self.ga.backward(gy4, saved)

    def g_s(self, y4, save=False):
        return self.gs.forward(y4, save)

    def g_s_backward(self, gx4, saved):
        return self.gs.backward(gx4, saved)

    def forward(self, x4, training=False, noise_y4=None, noise_z4=None):
        """entropy_estimator (anchors/model.py:97-106) + g_s(y_hat), eval mode."""
        if training:
            raise NotImplementedError("cheng2020 runs eval-mode forwards only (attack path)")
        N = self.N
        y4, _ = self.ga.forward(x4)
        z4 = self.ha.forward(y4)
        zh, zlik, zsum = K.eb_likelihood(z4, N, self.eb, False, None)
        params = self.hs.forward(zh)
        y_hat4 = K.round_(y4)
        ctx = self.ctx.forward(y_hat4)
        gp = self.ep.forward(torch.cat((params, ctx), dim=1))   # channel concat of nChw4c tensors
        c4 = (N + 3) // 4
        scales4 = gp[:, :c4].contiguous()
        means4 = gp[:, c4:].contiguous()
        _, ylik, ysum = K.gc_likelihood(y4, N, scales4, means4, False, None)
        xh, _ = self.gs.forward(y_hat4)
        return {"x_hat4": xh, "y4": y4, "y_hat4": y_hat4, "z4": z4, "z_hat4": zh, "scales4": scales4,
                "means4": means4, "lik4": {"y": ylik, "z": zlik}, "sumlog": ysum + zsum}

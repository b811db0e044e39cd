"""Autoregressive entropy coding of the context models (mbt2018 'context', cheng2020):
ar_coding.ArCoder on csrc/ica_ar.hip + the incremental host rANS decoder, and net.compress / decompress.

Checks (parity vs the oracle restatement of CompressAI's _compress_ar, oracle/entropy_coding.py; CompressAI's own
bitstreams are not available here: parity unpinned beyond that restatement):
  * the symbol / CDF-row streams of the HIP encoder equal the oracle's on the same (y, params) inputs, position-
    major, and the encoder's y_hat matches (the oracle sums in torch's order, the kernel in its own: the means
    agree to fp32 rounding, so the symbols, rounded from y - mean, are the same unless y - mean sits within ~1e-6
    of a half-integer; the seeds here have none);
  * decode(encode) restores the symbols and y_hat bit for bit (the decoder recomputes every mean on the same
    kernel), on a batch of images with different content;
  * net.compress / net.decompress on mbt2018 q1 and cheng2020 q1: the decoded reconstruction is
    clamp(g_s(y_hat)) of the encoder's y_hat, bit for bit; the y bitstream's size is sane against the eval
    forward's likelihood estimate."""
import pytest
import torch

from oracle import codec as oc
from oracle import entropy_coding as oe

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def rnd(shape, seed, lo=0.0, hi=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(shape, generator=g) * (hi - lo) + lo


def _coder(P, M):
    from imagecompression_adversarial_amd.ar_coding import ArCoder
    sd = {k: v.to(DEV) for k, v in P.items() if k.startswith(("context_prediction", "entropy_parameters"))}
    return ArCoder(sd, M, oe.get_scale_table().to(DEV))


@pytest.mark.parametrize("model,q,H,W", [("cheng2020", 1, 3, 5), ("context", 5, 4, 4)])
def test_ar_encode_vs_oracle(model, q, H, W):
    from imagecompression_adversarial_amd import hip_ops as K
    P = oc.perturb_params(oc.init_params(model, q, seed=0), seed=1)
    M = oc.model_channels(model, q)[1]
    y = rnd((2, M, H, W), 5, -6.0, 6.0)
    params = rnd((2, 2 * M, H, W), 6, -2.0, 2.0)
    ar = _coder(P, M)
    sym, idx, yhat4 = ar.encode(K.to_nc4(y.to(DEV)), K.to_nc4(params.to(DEV)))
    rs, ri, ryh = oe.compress_ar_symbols(P, y, params, oe.get_scale_table())
    assert torch.equal(sym.cpu(), rs), int((sym.cpu() != rs).sum())
    assert torch.equal(idx.cpu(), ri), int((idx.cpu() != ri).sum())
    yh = K.from_nc4(yhat4, M).cpu()
    assert float((yh - ryh).abs().max()) <= 1e-5 * float(ryh.abs().max())
    assert int(ri.min()) >= 0 and len(set(ri.flatten().tolist())) > 4   # several CDF rows in use


def test_ar_roundtrip_bitexact():
    from imagecompression_adversarial_amd import entropy_coding as EC_
    from imagecompression_adversarial_amd import hip_ops as K
    P = oc.perturb_params(oc.init_params("cheng2020", 1, seed=0), seed=2)
    M, B, H, W = 128, 3, 4, 6
    y = torch.cat([rnd((1, M, H, W), 10 + b, -3.0 * (b + 1), 3.0 * (b + 1)) for b in range(B)])
    params = rnd((B, 2 * M, H, W), 7, -1.0, 1.0)
    ar = _coder(P, M)
    p4 = K.to_nc4(params.to(DEV))
    sym, idx, yhat4 = ar.encode(K.to_nc4(y.to(DEV)), p4)
    tab = EC_.Tables(*EC_.gc_tables(oe.get_scale_table()))
    strings = EC_.encode_batch(sym, idx, tab)
    assert len(strings) == B and all(len(s) > 8 for s in strings)
    yhat_dec = ar.decode(strings, p4, tab)
    assert torch.equal(yhat_dec, yhat4)
    # and a corrupt stream is an error, not garbage
    with pytest.raises(RuntimeError):
        ar.decode([strings[0][:8]] + strings[1:], p4, tab)


def _net(model, q):
    from imagecompression_adversarial_amd import codec
    P = oc.perturb_params(oc.init_params(model, q, seed=0), seed=1)
    P["g_a.6.weight"] = P["g_a.6.weight"] * 20.0   # latents of a few units: real rates
    net = codec.mbt2018(q) if model == "context" else codec.cheng2020_anchor(q)
    sd = net.state_dict()
    sd.update({k: v.reshape(sd[k].shape) for k, v in P.items() if k in sd})
    net.load_state_dict(sd)
    net = net.to(DEV).eval()
    assert net.update() is True
    return net


@pytest.mark.parametrize("model,q", [("context", 1), ("cheng2020", 1)])
def test_context_model_compress_decompress(model, q):
    import math

    from imagecompression_adversarial_amd import codec
    from imagecompression_adversarial_amd import hip_ops as K
    net = _net(model, q)
    x = rnd((2, 3, 128, 192), 40, 0.0, 1.0).to(DEV)
    comp = net.compress(x)
    y_strings, z_strings = comp["strings"]
    assert len(y_strings) == 2 and len(z_strings) == 2 and tuple(comp["shape"]) == (2, 3)
    dec = net.decompress(comp["strings"], comp["shape"])
    # the encoder's own y_hat, through g_s
    ck = net.kernels()
    with torch.no_grad():
        y4, _ = ck.ga.forward(K.to_nc4(x))
        z4 = ck.ha.forward(y4)
        eb = net.entropy_bottleneck
        med = eb._get_medians().detach().reshape(-1).contiguous()
        from imagecompression_adversarial_amd import entropy_coding as EC_
        zs, _ = EC_.eb_symbols(z4, net.N, med)
        z_hat4 = EC_.dequantize(zs, 2, net.N, 2, 3, medians=med, device=x.device)
        p4 = ck.hs.forward(z_hat4)
        _, _, yhat4 = codec._ar_coder(net).encode(y4, p4)
        xh4, _ = ck.gs.forward(yhat4)
    assert torch.equal(dec["x_hat"], K.from_nc4(xh4, 3).clamp_(0, 1))
    # rate sanity: the eval forward's likelihood estimate (its context runs on round(y), the coder's on the coded
    # y_hat, so the two rates differ by the context mismatch, not by more than 2x)
    res = ck.forward(K.to_nc4(x))
    bits = -float(torch.log2(K.from_nc4(res["lik4"]["y"], net.M).clamp_min(1e-9)).sum())
    got = 8 * sum(len(s) for s in y_strings)
    assert math.isfinite(bits) and 0.5 * bits < got < 2.0 * bits + 1024, (got, bits)


def test_context_model_scale_table_update_rebuilds_coder():
    """update_scale_table(new, force=True) replaces the GaussianConditional's scale_table buffer; the cached ArCoder
    must follow it (its CDF-row indexes point into that table), so that a stream compressed after the update decodes
    in a freshly built model holding the same new table (the coder was keyed on parameters only)."""
    from imagecompression_adversarial_amd import codec
    net = _net("context", 1)
    x = rnd((1, 3, 128, 128), 41, 0.0, 1.0).to(DEV)
    net.compress(x)   # builds and caches the coder on the default table
    coarse = oe.get_scale_table()[::3].tolist()   # a shorter table: stale indexes would run past its CDFs
    assert net.gaussian_conditional.update_scale_table(coarse, force=True)
    assert codec._ar_coder(net).table.numel() == len(coarse)
    comp = net.compress(x)
    fresh = _net("context", 1)
    fresh.gaussian_conditional.update_scale_table(coarse, force=True)
    a = fresh.decompress(comp["strings"], comp["shape"])["x_hat"]
    b = net.decompress(comp["strings"], comp["shape"])["x_hat"]
    assert torch.equal(a, b)

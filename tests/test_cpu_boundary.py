"""CPU-side checks of the C-ABI boundary and the host mirror of the reference interface
(no GPU compute): the library loads and exports every symbol include/ica_hip.h declares;
the CLI keeps the reference flags and defaults (coder.py:166-220); image I/O rounding."""
import os
import re

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(REPO, "include", "ica_hip.h")).read()
    return sorted(set(re.findall(r"^(?:int|long|size_t)\s+(ica_\w+)\s*\(", txt, re.M)))


def test_library_exports_header_symbols():
    from imagecompression_adversarial_amd import _lib
    L = _lib.lib()
    syms = header_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    # every binding the Python layer declares is in the header too
    assert set(_lib.exported_symbols()) <= set(syms)


def header_prototypes():
    """name -> list of argument classes ('p' pointer / stream, 'i' int, 'l' long, 'f' float, 'z' size_t) and the
    return class, parsed from every `int|long|size_t ica_*(...)` prototype of include/ica_hip.h."""
    txt = open(os.path.join(REPO, "include", "ica_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", " ", txt, flags=re.S)
    out = {}
    for ret, name, args in re.findall(r"^(int|long|size_t)\s+(ica_\w+)\s*\(([^)]*)\)\s*;", txt, re.M):
        cls = []
        a = " ".join(args.split())
        if a not in ("", "void"):
            for arg in a.split(","):
                arg = arg.strip()
                if "*" in arg or arg.startswith("hipStream_t"):
                    cls.append("p")
                else:
                    typ = arg.rsplit(" ", 1)[0].replace("const ", "").strip()
                    cls.append({"int": "i", "long": "l", "float": "f", "size_t": "z"}[typ])
        out[name] = (cls, {"int": "i", "long": "l", "size_t": "z"}[ret])
    return out


def _ctype_class(t):
    import ctypes as C
    return {C.c_void_p: "p", C.c_int: "i", C.c_long: "l", C.c_float: "f", C.c_size_t: "z"}[t]


def test_bindings_match_header_prototypes():
    """Every ctypes binding in _lib._SIGS has the argument count, per-argument class (pointer / int / long /
    float / size_t) and return class of its include/ica_hip.h prototype: a stale binding or header fails here."""
    from imagecompression_adversarial_amd import _lib
    protos = header_prototypes()
    assert set(protos) == set(header_symbols())
    for name, args in _lib._SIGS.items():
        assert name in protos, name
        want, ret = protos[name]
        got = [_ctype_class(t) for t in args]
        assert got == want, (name, "".join(got), "".join(want))
        assert _ctype_class(_lib._RESTYPES.get(name, _lib._i)) == ret, name


def test_integration_snippet_matches_header():
    """The ctypes stub INTEGRATION.md shows a maintainer (`lib.<name>.argtypes = [...]`) declares each entry point
    exactly as include/ica_hip.h does."""
    doc = open(os.path.join(REPO, "INTEGRATION.md")).read()
    protos = header_prototypes()
    decl = re.findall(r"lib\.(ica_\w+)\.argtypes\s*=\s*\[([^\]]*)\]", doc)
    assert len(decl) >= 2
    letter = {"P": "p", "I": "i", "F": "f", "L": "l", "Z": "z"}
    for name, lst in decl:
        got = [letter[x.strip()] for x in lst.split(",") if x.strip()]
        assert got == protos[name][0], (name, "".join(got), "".join(protos[name][0]))
    # every call of a declared entry point in the snippet passes as many arguments as the prototype takes
    ncalls = 0
    for name, _ in decl:
        for mt in re.finditer(r"lib\.%s\(" % name, doc):
            depth, n, j = 1, 0, mt.end()
            empty = doc[j] == ")"
            while depth:
                ch = doc[j]
                depth += ch in "(["
                depth -= ch in ")]"
                n += ch == "," and depth == 1
                j += 1
            n = 0 if empty else n + 1
            assert n == len(protos[name][0]), (name, n, len(protos[name][0]))
            ncalls += 1
    assert ncalls >= len(decl)


def test_no_oracle_import_in_product():
    pkg = os.path.join(REPO, "imagecompression_adversarial_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(root, f)).read()
                assert "from oracle" not in src and "import oracle" not in src, f


def test_cli_flags_and_defaults():
    from imagecompression_adversarial_amd import coder
    a = coder.config().parse_args([])
    assert (a.model, a.metric, a.quality, a.steps, a.noise, a.epsilon, a.lr_attack, a.att_metric, a.random,
            a.clamp, a.device) == ("hyper", "ms-ssim", 3, 1001, 1e-4, 16.0, 0.01, "L2", 1, True, "cuda:0")
    a = coder.config().parse_args(["-m", "hyper", "-metric", "mse", "-q", "1", "-s", "x.png", "--no-clamp"])
    assert (a.model, a.metric, a.quality, a.source, a.clamp) == ("hyper", "mse", 1, "x.png", False)


def test_read_write_image_roundtrip(tmp_path):
    from PIL import Image
    from imagecompression_adversarial_amd import coder
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, size=(50, 70, 3), dtype=np.uint8)
    p = tmp_path / "a.png"
    Image.fromarray(img).save(p)
    x, H, W = coder.read_image(str(p))
    assert x.shape == (1, 3, 64, 128) and (H, W) == (50, 70)
    assert float(x[:, :, 50:, :].abs().max()) == 0.0 and float(x[:, :, :, 70:].abs().max()) == 0.0
    q = tmp_path / "b.png"
    coder.write_image(x, str(q), H, W)
    assert np.array_equal(np.array(Image.open(q)), img)


def test_write_image_round_half_even(tmp_path):
    from PIL import Image
    from imagecompression_adversarial_amd import coder
    # x*255 = 0.5, 1.5, 2.5 -> np.round half-to-even -> 0, 2, 2 (coder.py:45)
    v = torch.tensor([0.5, 1.5, 2.5, 253.5], dtype=torch.float64) / 255.0
    x = v.float().view(1, 1, 1, 4).repeat(1, 3, 1, 1)
    q = tmp_path / "c.png"
    coder.write_image(x, str(q))
    got = np.array(Image.open(q))[0, :, 0]
    ref = np.round(x[0, 0, 0].numpy() * 255.0).astype(np.uint8)  # float32 path as coder.py:45
    assert np.array_equal(got, ref)


def test_model_state_dict_keys():
    from imagecompression_adversarial_amd import codec
    m = codec.bmshj2018_hyperprior(1)
    keys = set(m.state_dict())
    for k in ("g_a.0.weight", "g_a.1.beta", "g_a.1.gamma", "g_a.1.beta_reparam.pedestal",
              "g_s.6.bias", "h_a.0.weight", "h_s.4.weight", "entropy_bottleneck._matrix0",
              "entropy_bottleneck._factor3", "entropy_bottleneck.quantiles", "gaussian_conditional.scale_table"):
        assert k in keys, k
    assert m.N == 128 and m.M == 192
    assert codec.bmshj2018_hyperprior(6).M == 320


@pytest.mark.parametrize("model,q", [("context", 3), ("context", 6), ("cheng2020", 6)])
def test_joint_model_keys_match_oracle(model, q):
    """mbt2018 / cheng2020 state dicts: every oracle parameter name exists with the same shape, and
    init_model builds them (anchors/model.py:74-77)."""
    from imagecompression_adversarial_amd.anchors import model as am
    from oracle import codec as oc
    m = am.init_model(model, q, "mse", pretrained=False)
    sd = m.state_dict()
    P = oc.init_params(model, q, seed=0)
    for k, v in P.items():
        assert k in sd, k
        assert sd[k].numel() == v.numel(), (k, tuple(sd[k].shape), tuple(v.shape))
    assert (m.N, m.M) == oc.model_channels(model, q)


def test_lr_schedule_matches_torch():
    from imagecompression_adversarial_amd.attack import _lr_table
    from oracle.attack import lr_schedule
    for steps in (1001, 100, 12, 3):
        assert _lr_table(steps, 0.01) == lr_schedule(steps, 0.01)


def test_aa_table_matches_torch_antialias_weights():
    """self_ensemble.aa_table (host logic) restates torch's float32 antialiased-bicubic weights: applying the
    tables on the CPU reproduces F.interpolate(..., antialias=True) to 2e-6."""
    import numpy as np
    import torch.nn.functional as F
    from imagecompression_adversarial_amd.self_ensemble import aa_table
    g = torch.Generator().manual_seed(0)
    for (H, W), sf in (((64, 96), 243 / 256), ((60, 91), 256 / 243), ((48, 40), 0.5)):
        x = torch.rand((1, 3, H, W), generator=g)
        ref = F.interpolate(x, scale_factor=sf, mode="bicubic", align_corners=False, antialias=True)
        Ho, Wo = ref.shape[2:]
        t = x.numpy()
        for axis, n_in, n_out in ((3, W, Wo), (2, H, Ho)):
            xmin, xsize, wt = aa_table(n_in, n_out, sf)
            t = np.moveaxis(t, axis, -1)
            o = np.zeros(t.shape[:-1] + (n_out,), np.float32)
            for i in range(n_out):
                acc = np.zeros(t.shape[:-1], np.float32)
                for k in range(xsize[i]):
                    acc = (acc + wt[i, k] * t[..., xmin[i] + k]).astype(np.float32)
                o[..., i] = acc
            t = np.moveaxis(o, -1, axis)
        assert float(np.abs(t - ref.numpy()).max()) < 2e-6


def test_header_compiles_as_c_and_cpp():
    """include/ica_hip.h is what a reference-side binding (ctypes / C / C++) reads: it must parse as C and C++."""
    import shutil
    import subprocess
    hdr = os.path.join(REPO, "include", "ica_hip.h")
    for cc, lang in (("gcc", "c"), ("g++", "c++")):
        if shutil.which(cc) is None:
            pytest.skip(f"{cc} not available")
        r = subprocess.run([cc, "-fsyntax-only", "-x", lang, hdr], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr


def test_old_format_checkpoint_conversion(tmp_path, capsys):
    """coder.load_model on an old-format checkpoint (coder.py:107-116): an anchors.balle.Image_coder state
    dict ("net." prefix, CDF buffers of the checkpoint's size) is converted, re-saved as ckpt + "new" with a
    "state_dict" key, and loaded; --eval on a training checkpoint reports epoch / step / lr (:138-146)."""
    import torch
    from imagecompression_adversarial_amd import coder
    from imagecompression_adversarial_amd.anchors import model as am
    src = am.init_model("hyper", 3, "mse", pretrained=False)
    coder._synthetic_init(src, seed=3)
    sd = src.state_dict()
    sd["entropy_bottleneck._quantized_cdf"] = torch.arange(128 * 7, dtype=torch.int32).reshape(128, 7)
    sd["entropy_bottleneck._offset"] = torch.full((128,), -3, dtype=torch.int32)
    sd["entropy_bottleneck._cdf_length"] = torch.full((128,), 7, dtype=torch.int32)
    old = {"net." + k: v for k, v in sd.items()}
    path = str(tmp_path / "old.pth")
    torch.save(old, path)
    args = coder.config().parse_args(["-m", "hyper", "-q", "3", "-metric", "mse", "-ckpt", path, "-device", "cpu"])
    net = coder.load_model(args, training=False)
    got = net.state_dict()
    for k, v in sd.items():
        assert torch.equal(got[k].cpu(), v), k
    new = torch.load(path + "new", weights_only=True)
    assert set(new) == {"state_dict"} and set(new["state_dict"]) == set(sd)
    # --eval on a training checkpoint
    args2 = coder.config().parse_args(["-m", "hyper", "-q", "3", "-metric", "mse", "--synthetic-weights",
                                       "-device", "cpu", "--adv"])
    net2, _, opt, aux, sch = coder.load_model(args2, training=True)
    torch.save({"epoch": 4, "step": 120, "state_dict": net2.state_dict(), "optimizer": opt.state_dict(),
                "aux_optimizer": aux.state_dict(), "lr_scheduler": sch.state_dict()}, str(tmp_path / "train.pth"))
    capsys.readouterr()
    args3 = coder.config().parse_args(["-m", "hyper", "-q", "3", "-metric", "mse", "-ckpt", str(tmp_path / "train.pth"),
                                       "-device", "cpu", "--eval", "--adv"])
    coder.load_model(args3, training=False)
    out = capsys.readouterr().out
    assert "Trained epoch 4" in out and "Trained step 120" in out and "Learning rate: 0.0001" in out


def test_b1_precision_code_documented():
    """prec = 3 (bf16 operands over fp32 activations on the k3 conv_downs, cheng2020 --precision bf16) is the
    hip_ops constant the C ABI header documents for ica_conv_args.prec."""
    import os
    from imagecompression_adversarial_amd import hip_ops as K
    assert (K.PREC_FP32, K.PREC_BF16, K.PREC_X6, K.PREC_B1) == (0, 1, 2, 3)
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "ica_hip.h")).read()
    assert "3: bf16 operands over fp32 tensors on the k3 conv_downs" in hdr
    from imagecompression_adversarial_amd.engine_cheng import _it, X6_IT
    assert _it(128) in X6_IT and _it(192) in X6_IT   # N = 128 and 192 both get the x6 / one-plane packs

"""CPU-side checks: the C-ABI library loads and exports every symbol include/endossl.h declares;
host logic (config defaults, schedulers, parameter layout, class weights) -- no GPU compute."""
import math
import os
import re
import subprocess

import numpy as np
import pytest
import torch

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, "include", "endossl.h")


def _declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t)\s+(es_\w+)\s*\(", txt, flags=re.M)))


def test_library_exports_every_declared_symbol():
    from endossl import _lib
    lib = _lib.load()
    decl = _declared()
    assert len(decl) >= 20
    for name in decl:
        assert hasattr(lib, name), name
    assert set(decl) == set(_lib.SIGNATURES), "python ctypes table out of sync with include/endossl.h"
    assert lib.es_abi_version() == _lib.ABI_VERSION
    assert lib.es_pack_entry_size() == 32 and lib.es_ema_entry_size() == 32


def test_library_is_gfx950_code_object():
    so = os.path.join(PKG, "endossl", "lib", "libendossl_hip.so")
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", so], capture_output=True, text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(so, "rb").read()
    assert b"gfx950" in blob


def test_arg_counts_match_header():
    from endossl import _lib
    txt = open(HEADER).read().replace("\n", " ")
    for name, (_, args) in _lib.SIGNATURES.items():
        m = re.search(r"\b" + name + r"\s*\(([^)]*)\)", txt)
        params = [p for p in m.group(1).split(",") if p.strip() and p.strip() != "void"]
        assert len(params) == len(args), name


def test_cpu_tensors_are_refused():
    from endossl import _lib
    with pytest.raises(_lib.EndosslCallError):
        _lib.ptr(torch.zeros(4))


def test_native_vit_layout_matches_timm_and_oracle():
    from endossl.vit import NativeViT, ViTConfig
    from oracle import ref
    m = NativeViT(ViTConfig(), seed=0)
    names = list(m.state_dict().keys())
    assert names == [n for n, _ in ref.param_shapes(ref.Cfg())]
    assert sum(p.numel() for p in m.parameters()) == 21_674_519
    for n, t in m.state_dict().items():
        assert t.data_ptr() >= m.flat.data_ptr()  # views into the flat buffer
        assert (t.data_ptr() - m.flat.data_ptr()) % 256 == 0
    # timm init: head zero, LN ones, linear std ~ .02
    sd = m.state_dict()
    assert float(sd["head.weight"].abs().max()) == 0.0
    assert float(sd["blocks.0.norm1.weight"].min()) == 1.0
    assert abs(float(sd["blocks.3.mlp.fc1.weight"].std()) - 0.02) < 0.002
    # loading a state_dict writes through to the flat buffer
    sd2 = {k: torch.full_like(v, 0.5) for k, v in sd.items()}
    m.load_state_dict(sd2)
    assert float(m.flat[m.offs["pos_embed"]]) == 0.5
    with pytest.raises(Exception):
        m(torch.zeros(1, 3, 224, 224))  # CPU: no fallback


def test_deepcopy_gives_independent_flat():
    from copy import deepcopy
    from endossl.vit import NativeViT, ViTConfig
    m = NativeViT(ViTConfig(img_size=64, dim=128, depth=2, heads=2), seed=1)
    e = deepcopy(m)
    assert e.flat.data_ptr() != m.flat.data_ptr()
    torch.testing.assert_close(e.flat, m.flat)
    e.flat.add_(1.0)
    assert float((e.flat - m.flat).abs().min()) > 0.5
    assert list(e.state_dict()) == list(m.state_dict())


def test_config_defaults_fill_missing_keys(tmp_path):
    from endossl.utils import get_config
    p = tmp_path / "c.yaml"
    p.write_text("DATA:\n BATCH_SIZE: 8\nMODEL:\n NAME: 'vit_small_patch16_224'\n MARGIN: None\nTRAIN:\n THRES: 0.7\n")
    c = get_config(str(p))
    assert c.DATA.BATCH_SIZE == 8 and c.TRAIN.THRES == 0.7
    assert c.MODEL.PRE_TRAIN_RESUME == "None" and c.TRAIN.IS_FREEZE is False  # missing in several ref configs
    assert c.MODEL.MARGIN == "None"  # PyYAML parses `None` as a string


def test_reference_configs_parse():
    from endossl.utils import get_config
    cdir = "/root/reference/code/configs"
    if not os.path.isdir(cdir):
        pytest.skip("reference configs only in the build container")
    for f in sorted(os.listdir(cdir)):
        c = get_config(os.path.join(cdir, f))
        assert "BATCH_SIZE" in c.DATA and "EMA_DECAY" in c.TRAIN


def test_step_scheduler_and_warmup():
    from endossl.lr_scheduler import StepLRScheduler, CosineLRScheduler

    class Opt:
        param_groups = [{"lr": 1e-3}, {"lr": 1e-3}]
    o = Opt()
    s = StepLRScheduler(o, decay_t=10, decay_rate=0.8, warmup_t=5, warmup_lr_init=5e-4, t_in_epochs=False)
    assert o.param_groups[0]["lr"] == 5e-4
    s.step_update(2)
    assert math.isclose(o.param_groups[0]["lr"], 5e-4 + 2 * (1e-3 - 5e-4) / 5)
    s.step_update(25)
    assert math.isclose(o.param_groups[1]["lr"], 1e-3 * 0.8 ** 2)
    o2 = Opt()
    o2.param_groups = [{"lr": 1e-3}]
    c = CosineLRScheduler(o2, t_initial=100, lr_min=5e-6, t_in_epochs=False)
    c.step_update(50)
    assert math.isclose(o2.param_groups[0]["lr"], 5e-6 + 0.5 * (1e-3 - 5e-6) * (1 + math.cos(math.pi * 0.5)))


def test_balanced_class_weights_match_sklearn_formula():
    from endossl.utils import balanced_class_weights
    y = np.concatenate([np.full(i + 1, i) for i in range(23)])
    w = balanced_class_weights(y)
    np.testing.assert_allclose(w, len(y) / (23 * np.bincount(y)), rtol=1e-6)


def test_class_weights_match_fixture(golden):
    from endossl.utils import balanced_class_weights
    d = golden("fixmatch_step_t0p7.npz")
    y = np.concatenate([np.full(i + 1, i) for i in range(23)])
    np.testing.assert_array_equal(balanced_class_weights(y), d["class_weights"])


def test_average_meter():
    from endossl.utils import AverageMeter
    m = AverageMeter()
    m.update(2.0, 4)
    m.update(4.0, 4)
    assert m.avg == 3.0 and m.count == 8


def test_vit_emb_layout_matches_reference_modelwemb(golden):
    """NativeViTEmb's state_dict = the reference ModelwEmb-style model's (names, shapes, order,
    BatchNorm1d buffers), on the CPU (no kernel calls)."""
    from endossl.comatch_model import NativeViTEmb
    from endossl.vit import ViTConfig
    d = golden("comatch_step_closed.npz")
    m = NativeViTEmb(ViTConfig(img_size=64, dim=128, depth=2, heads=2, num_classes=23, head="emb",
                               low_dim=int(d["L"])), seed=0)
    sd = m.state_dict()
    ref_keys = [k[5:] for k in d.files if k.startswith("init/")]
    assert list(sd.keys()) == ref_keys
    for k in ref_keys:
        assert tuple(sd[k].shape) == d["init/" + k].shape, k
        assert sd[k].dtype == {"float32": torch.float32, "int64": torch.int64}[str(d["init/" + k].dtype)], k
    m.load_state_dict({k: torch.tensor(d["init/" + k]) for k in ref_keys})
    assert torch.equal(m.fc[4].weight.detach() if hasattr(m.fc, "__getitem__") else
                       m.fc._modules["4"].weight.detach(), torch.tensor(d["init/fc.4.weight"]))
    import copy
    e = copy.deepcopy(m)
    assert torch.equal(e.state_dict()["fc.3.running_var"], sd["fc.3.running_var"])


def test_build_model_routes_comatch():
    from endossl.build import build_model
    from endossl.comatch_model import NativeViTEmb
    from endossl.utils import AttrDict, with_defaults
    cfg = with_defaults(AttrDict(MODEL=AttrDict(NAME="vit_tiny_test", NUM_CLASSES=23, TYPE_SEMI="CoMatch", LOW_DIM=16),
                                 TRAIN=AttrDict(IS_SSL=True), DATA=AttrDict(IMG_SIZE=64)))
    m = build_model(cfg)
    assert isinstance(m, NativeViTEmb) and m.cfg.low_dim == 16 and m.cfg.head == "emb"


def test_conformer_layout_matches_reference_state_dict(golden):
    """NativeConformer's state_dict = the reference Conformer's (names, order, shapes), taken from
    the fixture the reference itself produced (tests/golden/make_golden.py gen_semiformer_step)."""
    from endossl.conformer import ConformerConfig, NativeConformer
    d = golden("semiformer_step.npz")
    keys = [k[5:] for k in d.files if k.startswith("init/")]
    m = NativeConformer(ConformerConfig(img_size=64, embed_dim=128, depth=6, heads=2, num_classes=23), seed=0)
    sd = m.state_dict()
    assert list(sd.keys()) == keys
    for k in keys:
        assert tuple(sd[k].shape) == tuple(d["init/" + k].shape), k
        assert sd[k].dtype == torch.from_numpy(d["init/" + k]).dtype, k
    m.load_state_dict({k: torch.tensor(d["init/" + k]) for k in keys})
    assert torch.equal(m.get_parameter("conv_trans_6.trans_block.mlp.fc2.weight"),
                       torch.tensor(d["init/conv_trans_6.trans_block.mlp.fc2.weight"]))
    # parameters are views of the flat buffer (one Adam + EMA sweep)
    p = m.get_parameter("conv1.weight")
    assert p.data_ptr() == m.flat.data_ptr() + 4 * m.offs["conv1.weight"]


def test_build_model_routes_conformer():
    from endossl.build import build_model
    from endossl.utils import AttrDict
    cfg = AttrDict(DATA=AttrDict(IMG_SIZE=224), MODEL=AttrDict(NAME="conformer", NUM_CLASSES=23, PRE_TRAIN_PATH="None"),
                   TRAIN=AttrDict())
    m = build_model(cfg)
    assert type(m).__name__ == "NativeConformer"
    assert m.cfg.dim == 384 and m.cfg.depth == 12 and m.cfg.heads == 6 and m.cfg.T == 197
    assert m.get_parameter("conv_cls_head.weight").shape == (23, 256)


def test_tn_big_grouped_prepare_layout():
    """es_gemm_tn_big_grouped_prepare is host code (no GPU): a ViT-S block's four weight gradients at the
    F1 token count get the same split count (target / 24 tiles), split-major workgroup ranges, slabs and
    bias partials carved from the workspace in problem order, and one reduce entry per slab set and per
    bias; a workspace one float short is refused."""
    import ctypes
    import struct

    from endossl import _lib
    from endossl.vit import _TNProblem
    lib = _lib.load()
    D, Hd, M = 384, 1536, 100864
    shapes = [(D, Hd), (Hd, D), (D, D), (3 * D, D)]
    tab = (_TNProblem * 4)()
    for k, (e, (N1, N2)) in enumerate(zip(tab, shapes)):
        e.dy, e.x, e.out, e.bias_out = 0x1000 * (k + 1), 0x100000 * (k + 1), 0x2000000 * (k + 1), 0x30000000 * (k + 1)
        e.M, e.N1, e.N2, e.ld1, e.ld2 = M, N1, N2, N1, N2
    need = lib.es_gemm_tn_big_grouped_workspace(ctypes.byref(tab), 4, 128)
    assert need == 5 * sum(N1 * N2 + N1 for N1, N2 in shapes)
    raw = ctypes.create_string_buffer(lib.es_gemm_tn_big_grouped_table_bytes(4))
    dims = (ctypes.c_int * 3)()
    base = 0x7000000000
    assert lib.es_gemm_tn_big_grouped_prepare(ctypes.byref(tab), 4, 128, ctypes.c_void_p(base), need, raw, dims) == 0
    assert list(dims)[0] == 5 * 24 and list(dims)[2] == 8
    off, wg = 0, 0
    for i, (N1, N2) in enumerate(shapes):
        a1, a2, P, PB, m, n1, n2, l1, l2, mchunk, wg0, nt, S, _ = struct.unpack_from("4Q6i4i", raw.raw, i * 72)
        assert (a1, a2, m, n1, n2) == (tab[i].dy, tab[i].x, M, N1, N2) and S == 5 and mchunk == 316 * 64
        assert P == base + 4 * off and PB == P + 4 * S * N1 * N2 and wg0 == wg and nt == (N1 // 384) * (N2 // 192)
        off += S * (N1 * N2 + N1)
        wg += S * nt
    assert lib.es_gemm_tn_big_grouped_prepare(ctypes.byref(tab), 4, 128, ctypes.c_void_p(base), need - 1, raw,
                                              dims) != 0


def test_resid_ln_entry_validates_before_any_launch():
    """es_gemm_nt_resid_ln refuses what its kernel cannot take before touching the GPU: any width but 384
    (ES_BAD_SHAPE), misaligned row strides (ES_BAD_SHAPE: the LDS-DMA moves 16-B row pieces), a null operand
    (ES_BAD_ARG)."""
    from endossl import _lib
    lib = _lib.load()
    p = 0x7000000000  # never dereferenced on these paths

    def rc(M=256, N=384, K=384, lda=384, ldc=384, ldaux=384, ldh=384, gamma=p):
        return lib.es_gemm_nt_resid_ln(p, lda, p, 384, None, p, ldc, p, ldaux, gamma, p, p, ldh, p, p, M, N, K, 1e-6,
                                       None)
    assert rc(N=768) == -1 and rc(K=768) == -1 and rc(M=0) == -1
    assert rc(lda=388) == -1 and rc(ldaux=386) == -1 and rc(ldc=385) == -1 and rc(ldh=385) == -1
    assert rc(gamma=None) == -2
    assert rc(gamma=p + 4) == -2  # a misaligned operand (16-B pieces)


INTEGRATION = os.path.join(ROOT, "INTEGRATION.md")


def _expand_doc_name(tok):
    """`es_x(_a / _b)y` -> es_xy, es_x_ay, es_x_by (the empty alternative included); other tokens as they are."""
    m = re.search(r"\(([^)]*)\)", tok)
    if not m:
        return [tok]
    alts = [""] + [a.strip() for a in m.group(1).split("/")]
    out = []
    for a in alts:
        out += _expand_doc_name(tok[:m.start()] + a + tok[m.end():])
    return out


def _doc_names():
    """Every es_* name INTEGRATION.md names inside backticks (groups expanded; `*` kept as a glob)."""
    names = set()
    for span in re.findall(r"`([^`\n]+)`", open(INTEGRATION).read()):
        for tok in re.findall(r"\bes_[A-Za-z0-9_*]+(?:\([^)]*\)[A-Za-z0-9_*]*)?", span):
            names.update(_expand_doc_name(tok))
    return names


def test_integration_doc_matches_header():
    """INTEGRATION.md names only entry points include/endossl.h declares, and names all of them (round-4
    verdict: the doc kept four entry points the knob pruning had removed)."""
    import fnmatch
    decl = set(_declared())
    doc = _doc_names()
    assert len(doc) > 50
    missing = [n for n in doc if not (fnmatch.filter(decl, n) if "*" in n else n in decl)]
    assert not missing, f"INTEGRATION.md names entry points the header does not declare: {sorted(missing)}"
    covered = {d for d in decl if any(fnmatch.fnmatch(d, n) if "*" in n else d == n for n in doc)}
    assert covered == decl, f"header entry points INTEGRATION.md does not document: {sorted(decl - covered)}"


def _package_sources():
    out = {}
    for base in (os.path.join(PKG, "endossl"), os.path.join(PKG, "csrc")):
        for f in sorted(os.listdir(base)):
            if f.endswith((".py", ".hip", ".cpp", ".h")):
                out[os.path.join(base, f)] = open(os.path.join(base, f)).read()
    out[os.path.join(ROOT, "bench.py")] = open(os.path.join(ROOT, "bench.py")).read()
    return out


def test_integration_doc_knobs_are_the_ones_the_code_reads():
    """The ENDOSSL_* variables INTEGRATION.md documents are exactly those the package and bench read
    (os.environ lookups), so a pruned knob cannot linger in the doc."""
    doc = set(re.findall(r"\bENDOSSL_[A-Z0-9_]+", open(INTEGRATION).read()))
    read = set()
    for txt in _package_sources().values():
        read.update(re.findall(r"environ(?:\.get)?[\(\[]\s*[\"'](ENDOSSL_[A-Z0-9_]+)", txt))
        read.update(re.findall(r"\(\"(ENDOSSL_[A-Z0-9_]+)\",\s*\"es_set_", txt))  # _lib.py's pin table
    assert len(read) >= 10, read
    assert doc == read, {"documented, not read": sorted(doc - read), "read, not documented": sorted(read - doc)}


def test_kernel_family_pins_refuse_removed_families():
    """Host-only setters (no GPU work): a pin to a kernel family that no longer exists returns ES_BAD_ARG and
    leaves the setting alone (round-4 advice: removed pins used to fall back to family 0 silently)."""
    from endossl import _lib
    lib = _lib.load()
    for setter, good, bad in (("es_set_gemm_variant", (-1, 0, 1, 2, 5, 6, 10, 11, 12), (3, 4, 7, 8, 9, 13, 21, -2)),
                              ("es_set_tn_variant", (-1, 0, 7), (1, 2, 5, 6, 8, 13)),
                              ("es_set_attn_bwd_variant", (0, 1, 2, 3, 4), (5, -1)),
                              ("es_set_conv_ring", (0, 3, 4), (1, 2, 5, -1)),
                              ("es_set_conv_dw_buf", (1, 0), (2, -1)),
                              ("es_set_conv_small", (128, 0, 64, 512), (-1, -5)),
                              ("es_set_bn_cs", (1, 0), (2, -1)),
                              ("es_set_bn_sum8", (0, 1), (2, -1))):
        fn = getattr(lib, setter)
        base = fn(good[0])
        for v in bad:
            assert fn(v) == -2, (setter, v)
            assert fn(good[0]) == good[0], (setter, v)  # unchanged by the refused pin
        for v in good:
            fn(v)
            assert fn(good[0]) == v, (setter, v)
        fn(base)

"""Benchmark: unlabeled images/sec of the FixMatch ViT-S/16 SSL step (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--scaling strong|weak]
  (N>1: launched by torch.distributed.run, one rank per GPU, RCCL over xGMI)

Workload F1 (BASELINE configs[1]; configs[2] at N > 1): FixMatch, ViT-Small/16, global batch B=64
labeled + mu*B = 448 unlabeled weak/strong pairs, 224x224x3, 23 classes, bf16 MFMA compute with
fp32 master weights.  Synthetic, HBM-resident inputs (seed 0): uint8 pixels whose ToTensor +
ImageNet Normalize (code/dataset.py:21-22,49-51) run inside the patch gather (--inputs f32:
host-normalised fp32 images).
Scaling (north_star / SURVEY.md §8(e)): "strong" (default) shards the global batch over the N ranks
(64/N labeled + 448/N pairs per GPU: the DDP average of per-rank means is the global-batch gradient);
"weak" gives every rank the full F1 batch.  The flat fp32 gradient's RCCL all-reduce is the only
exchange.  One step = weak forward + train forward/backward + fused losses + grad all-reduce +
Adam/EMA sweep (code/fixmatch.py:91-131) -- nothing skipped.  Eager launches (--graph on replays
the forward/backward as one captured hipGraph, FixMatch.use_graph: measured slower here).  At N > 1
with strong scaling the line also carries `weak_scaling`: the same step timed with a full batch per
rank (configs[2] as DDP would run it).

Reported beside it:
  roofline      the dominant kernel (the most GPU time per step: rocprofv3, profiles/r04e_summary.md) = a
                transformer block's four weight-gradient GEMMs as ONE split-K launch (es_gemm_tn_big_grouped:
                gemm_tn_big_grouped_kernel + its reduce), timed live by events the kernels stamp themselves
                (hipExtLaunchKernelGGL) on the side stream they run on, at the CU-share-sized launches of blocks
                10..1: algorithmic 2*M*(384*1536 + 1536*384 + 384*384 + 1152*384) FLOP per launch (M = train
                tokens) vs the bf16 dense MFMA peak 2516.6 TFLOP/s; `isolated` = the same launch with the second
                stream off.  traffic = HBM bytes of that launch inside the F1 step from rocprofv3 --pmc
                FETCH_SIZE (x2, gfx950) / WRITE_SIZE passes over this bench (scripts/gpu_pmc_step.sh ->
                profiles/pmc_traffic.json, labelled with the library build it was measured on).
  step_tflops   algorithmic 18.247 TFLOP per F1 step / step time.  The engine skips
                the last block's non-CLS rows after its qkv GEMM (their outputs never reach the head;
                Engine.PRUNE_LAST), so it executes fewer FLOPs than that: `executed_step_tflop`.
  mfma_util     the step's MFMA-busy SIMD-cycles from committed rocprofv3 --pmc passes
                (profiles/<tag>_step_counters.json) over this run's step time; marked as measured on this
                library build or as an estimate from another one (sha256 of libendossl_hip.so).
  cpu_baseline  the oracle (CPU fp32 restatement pinned to the reference, kind "port") on every host core the
                job may use, rank 0, N=1, on a bounded sample: B=16, mu=7 (112 unlabeled images per step),
                one warm-up step then one timed step (~15 s each on the GPU box's 16 threads).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)
PEAK_BF16_TFLOPS = 256 * 2.4e9 * 4096 / 1e12  # 2516.6 dense (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md §HBM; ~6300 achievable)
STEP_TFLOP_F1 = 18.247  # fwd 960 imgs + bwd 512 imgs, 9.197 GFLOP/img fwd


def vit_s_pruned_tflop(n_fwd, n_bwd):
    """FLOPs the last block does NOT execute with Engine.PRUNE_LAST / PRUNE_Q (ViT-S/16 at 224^2):
    for the 196 non-CLS tokens of each image, projection + fc1 + fc2 (2*D*(D + 2*Hd)) and their
    attention queries (4*T*64*H) -- forward over n_fwd images, backward (2x) over n_bwd -- and the Q
    projection (2*D*D): forward over n_fwd, its weight gradient (1x; the data gradient still runs)
    over n_bwd."""
    from endossl.vit import Engine
    D, Hd, T, H = 384, 1536, 197, 6
    per_img = (T - 1) * (2 * D * (D + 2 * Hd) + 4 * T * 64 * H)
    q = (T - 1) * 2 * D * D
    return (per_img * (n_fwd + 2 * n_bwd) + (q * (n_fwd + n_bwd) if Engine.PRUNE_Q else 0)) / 1e12


def synth_u8(n, size, gen, device):
    return torch.randint(0, 256, (n, 3, size, size), generator=gen, dtype=torch.uint8, device=device)


def synth_images(n, size, gen, device):
    u8 = synth_u8(n, size, gen, device)
    x = u8.float().div_(255.0)
    m = torch.tensor(MEAN, device=device).view(1, 3, 1, 1)
    s = torch.tensor(STD, device=device).view(1, 3, 1, 1)
    return x.sub_(m).div_(s)


def host_cpus():
    """CPUs this process may actually use: os.cpu_count() capped by the affinity mask and the cgroup
    CPU quota (a GPU box shows the whole machine's 256 threads but grants a share of them)."""
    n = os.cpu_count() or 1
    info = {"os.cpu_count": n}
    try:
        aff = len(os.sched_getaffinity(0))
        info["affinity"] = aff
        n = min(n, aff)
    except (AttributeError, OSError):
        pass
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            txt = open(path).read().split()
            if path.endswith("cpu.max") and txt[0] != "max":
                q = int(txt[0]) / int(txt[1])
            elif path.endswith("quota_us") and int(txt[0]) > 0:
                q = int(txt[0]) / int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            else:
                continue
            info["cgroup_quota"] = q
            n = min(n, max(1, int(q)))
            break
        except (OSError, ValueError, IndexError):
            continue
    return n, info


def host_input_run(tr, B, MU, steps, dev):
    """F1 steps whose batches come from the native host input path: decoded
    RGB frames -> the reference's TransformFixMatch / labeled transforms on the granted host threads
    (csrc/host_aug.cpp) -> pinned uint8 -> side-stream H2D copy, double-buffered against the step."""
    import numpy as np

    from endossl import host_aug
    threads, _ = host_cpus()
    g = np.random.default_rng(7)
    base = g.integers(0, 256, (60, 80, 3), dtype=np.uint8)
    srcs = [host_aug.resize_bilinear(base ^ np.uint8(i * 29 % 256), (500, 375)) for i in range(64)]
    lab = host_aug.HostBatcher(srcs, batch=B, size=224, kind="labeled", seed=1, threads=threads, device=dev)
    unl = host_aug.HostBatcher(srcs, batch=B * MU, size=224, kind="fixmatch", seed=2, threads=threads, device=dev)
    y = torch.randint(0, 23, (B,), device=dev)

    def one():
        (x,) = lab.next()
        uw, us = unl.next()
        return tr.step(((x, y), ((uw, us), None)))

    for _ in range(2):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t1 = time.perf_counter()  # the host transforms alone, same threads (what bounds the fed step)
    host_aug.transform_batch(srcs[:32] * 4, 224, "fixmatch", seed=3, threads=threads)
    pairs = 128 / (time.perf_counter() - t1)
    return {"value": round(B * MU * steps / dt, 2), "unit": "unlabeled images/s", "ms_per_step": round(dt / steps * 1e3, 3),
            "host_threads": threads, "host_fixmatch_pairs_per_s": round(pairs, 1),
            "source": "synthetic decoded RGB 500x375 frames (64), IS_CROP, S=224; decode not timed"}


def cpu_baseline(B=16, MU=7, steps=3, warmup=1):
    """Oracle (pinned CPU restatement) FixMatch step on every host core this process may use -- a
    reported baseline (torch.set_num_threads(os.cpu_count()), capped by the CPU share the
    box grants: more threads than cores only oversubscribes).  Default: a bounded sample of the F1 step,
    B=16, mu=7 (112 unlabeled images), one warm-up step (thread pools, first-touch of the allocator's pages)
    then the mean of three timed steps (BASELINE.md's plan), ~65 s in all; --cpu-batch 64 runs the full F1
    batch (~100 GB of fp32 autograd activations, ~55 s per step)."""
    from oracle import ref
    threads, cpu_info = host_cpus()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    cfg = ref.Cfg()
    params = ref.random_params(cfg, seed=0)
    fm = ref.FixMatchRef(params, cfg, class_weights=None, thres=0.95, lambda_u=1.0)
    g = torch.Generator().manual_seed(0)
    x = synth_images(B, 224, g, "cpu")
    y = torch.randint(0, 23, (B,), generator=g)
    uw = synth_images(B * MU, 224, g, "cpu")
    us = synth_images(B * MU, 224, g, "cpu")
    for _ in range(warmup):
        fm.step(x, y, uw, us)
        print(f"cpu_baseline: warm-up step done on {threads} threads", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    for i in range(steps):
        fm.step(x, y, uw, us)
        print(f"cpu_baseline: step {i + 1}/{steps}", file=sys.stderr, flush=True)
    dt = (time.perf_counter() - t0) / steps
    used = torch.get_num_threads()
    torch.set_num_threads(prev)
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    mem = "unknown"
    try:
        for line in open("/proc/meminfo"):
            if line.startswith("MemTotal"):
                mem = f"{int(line.split()[1]) / 2**20:.0f} GiB"
                break
    except (OSError, ValueError, IndexError):
        pass
    return {"value": round(B * MU / dt, 3), "unit": "unlabeled images/s", "cores": used,
            "kind": "port",
            "sample": f"oracle FixMatch step, ViT-S/16 224^2 fp32, B={B} mu={MU} ({B * MU} unlabeled imgs/step"
                      f"{'; the full F1 batch' if B == 64 else '; a reduced batch, not the F1 B=64'}), "
                      f"{warmup} warm-up + {steps} timed steps, {dt:.2f} s/step, cpu='{cpu}', host CPUs {cpu_info}, "
                      f"host RAM {mem} (the job may use at most ~270 GiB of it), torch.get_num_threads()={used}"}


def lib_sha256():
    """sha256 of the device library this process loads (ties committed counter files to a build)."""
    import hashlib
    from endossl import _lib
    try:
        with open(_lib.LIB_PATH, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()
    except OSError:
        return None


def step_counters():
    """The committed step-level counter summary (scripts/gpu_step_counters.sh -> profiles/<tag>_step_counters.json,
    the newest tag): MFMA-busy SIMD-cycles and HBM bytes of one F1 step, measured by rocprofv3 --pmc passes over
    this bench."""
    pdir = os.path.join(ROOT, "profiles")
    cands = sorted(f for f in os.listdir(pdir) if f.endswith("_step_counters.json"))
    if not cands:
        return None, None
    with open(os.path.join(pdir, cands[-1])) as f:
        return json.load(f), "profiles/" + cands[-1]


def pmc_traffic(kernel_substr):
    """Per-launch HBM bytes of the dominant kernel from the committed rocprofv3 --pmc summary
    (profiles/pmc_traffic.json: FETCH_SIZE x2 (gfx950 half-count correction) + WRITE_SIZE, KiB->B)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None, None
    try:
        d = json.load(open(p))
        for k, v in d.get("kernels", {}).items():
            if kernel_substr in k:
                build = ("measured on this library build" if v.get("lib_sha256") and v.get("lib_sha256") == lib_sha256()
                         else "measured on another library build: an estimate for this one")
                return v.get("hbm_bytes_per_launch"), f"committed profiles/pmc_traffic.json entry '{k}', {build}"
    except (OSError, ValueError):
        return None, None
    return None, None


def conformer_step_tflop(cfg, n_images):
    """Algorithmic FLOP of one SemiFormer step: 3x the Conformer forward (forward + backward, every
    row carries gradient through BatchNorm) over n_images.  Forward per image: every conv
    (2 * Cout * Cin * k^2 per output pixel), the transformer blocks (24 D^2 per token in the linears
    + 4 T D per token in attention) and the FCU 1x1 convs, at the Conformer's own resolutions."""
    S = cfg.img_size
    fl = 2 * 64 * 3 * 49 * (S // 2) ** 2                      # stem conv1
    hw = cfg.stem ** 2

    def block(inp, outp, stride, res, hw_in):
        med = outp // 4
        hw_out = hw_in // (stride * stride)
        f = 2 * med * inp * hw_in + 2 * med * med * 9 * hw_out + 2 * outp * med * hw_out
        return f + (2 * outp * inp * hw_out if res else 0), hw_out

    f, hw = block(64, cfg.s1, 1, True, hw)
    fl += f + 2 * cfg.dim * 64 * cfg.dw ** 2 * cfg.np                       # conv_1, trans_patch_conv
    tb = cfg.T * (24 * cfg.dim ** 2 + 4 * cfg.T * cfg.dim)                  # one transformer block
    fl += tb
    for _, inp, outp, res, stride, dw, last in cfg.stages():
        f, hw = block(inp, outp, stride, res, hw)
        med = outp // 4
        fl += f + 2 * cfg.dim * med * hw + tb + 2 * med * cfg.dim * cfg.np   # cnn_block, FCUDown, block, FCUUp
        f, hw2 = block(outp, outp, 2 if last else 1, last, hw)
        fl += f
        hw = hw2
    return 3 * fl * n_images / 1e12


def run_secondary(args):
    """--workload c1 / s1: the other BASELINE configs on one GPU (step time and unlabeled images/s).
    c1: CoMatch ViT-S/16, B=64, mu=7, 65,536-entry bank, EMA 0.999 (configs[3], single-GPU leg);
    s1: SemiFormer on build.py's Conformer-Ti at 224^2, B=24, mu=7 (configs[4] names a ViT-B/384
    Conformer that build.py cannot construct -- SURVEY.md §8(a) a20)."""
    from endossl import dist
    from endossl.utils import AttrDict
    rank, world, local = dist.init_from_env()
    _check_world(args, world)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    map_dtype = None  # the Conformer's CNN map dtype (S1)
    if args.workload == "c1":
        from endossl.comatch import CoMatch
        from endossl.comatch_model import NativeViTEmb
        from endossl.vit import ViTConfig
        B, MU, L, Q = 64, 7, 64, 65536
        model = NativeViTEmb(ViTConfig(head="emb", low_dim=L), seed=0)
        tr = CoMatch(model, device=dev)
        cfg = AttrDict(DATA=AttrDict(BATCH_SIZE=B, MU=MU, IMG_SIZE=224, TARGET_NAME="target"),
                       MODEL=AttrDict(NAME="vit_small_patch16_224", NUM_CLASSES=23, LOW_DIM=L, TYPE_SEMI="CoMatch"),
                       TRAIN=AttrDict(IS_FREEZE=False, USE_EMA=True, EMA_DECAY=0.999, BASE_LR=1e-3, EVAL_STEP=1,
                                      CLS_WEIGHT=False, THRES=0.95, T=1.0, LAMBDA_U=2.0, LAMBDA_C=2.0, EPOCHS=1,
                                      WARMUP_EPOCHS=0, DECAY_EPOCHS=10, WARMUP_LR=5e-4, LR_DECAY=0.8, SCH_NAME="const"))
        tr.get_dataloader((None, None), None)
        tr.get_config(cfg)
        tr.set_queue_size(Q)
        # a populated bank (as after earlier epochs): unit features, softmax class rows
        tr.queue_feats.copy_(torch.nn.functional.normalize(torch.randn(Q, L, generator=g, device=dev), dim=1))
        tr.queue_probs.copy_(torch.softmax(torch.randn(Q, 23, generator=g, device=dev) * 3, 1))
        x, y = synth_images(B, 224, g, dev), torch.randint(0, 23, (B,), generator=g, device=dev)
        batch = ((x, y), tuple(synth_images(B * MU, 224, g, dev) for _ in range(3)), None)
        batch = (batch[0], (batch[1], None))
        unl, tfl = B * MU, 3 * 9.197e9 * (B + 3 * B * MU) / 1e12 + 2 * (B * MU) * Q * (L + 23) / 1e12
        from endossl.vit import Engine
        exe = tfl - (vit_s_pruned_tflop(B + 3 * B * MU, B + 3 * B * MU) if Engine.PRUNE_LAST
                     else 0.0)
        desc = (f"C1: CoMatch ViT-S/16 step, B={B} + 3 x mu*B={B * MU} (weak, strong0, strong1), 224^2, L={L}, "
                f"bank Q={Q} (memory smoothing over all Q rows), EMA 0.999, lambda_u=lambda_c=2")
    elif args.workload == "p0":
        # BASELINE configs[0]: the supervised baseline (code/supervised.py:111-138 plain path) -- the
        # reference runs it on CPU as plumbing; here the native ResNet-18 step on the GPU
        from endossl.resnet import NativeResNet, ResNetConfig
        from endossl.supervised import SupLearning
        B = args.batch if args.batch != 64 else 16
        model = NativeResNet(ResNetConfig(num_classes=23), seed=0)
        tr = SupLearning(model, device=dev)
        if args.graph != "auto":  # auto: SupLearning's default (the forward / backward replayed as one hipGraph)
            tr.use_graph = args.graph == "on"

        class _DS:
            df = None
        tr.get_dataloader(type("DL", (list,), {"dataset": _DS()})(), None, None)
        tr.get_config(AttrDict(DATA=AttrDict(BATCH_SIZE=B, IMG_SIZE=224, TARGET_NAME="target"),
                               MODEL=AttrDict(NAME="resnet18", NUM_CLASSES=23, MARGIN="None", IS_TRIPLET=False),
                               TRAIN=AttrDict(USE_EMA=True, EMA_DECAY=0.999, BASE_LR=1e-3, CLS_WEIGHT=False, EPOCHS=1,
                                              WARMUP_EPOCHS=0, DECAY_EPOCHS=10, WARMUP_LR=5e-4, LR_DECAY=0.8,
                                              SCH_NAME="const")))
        tr.class_weights = torch.linspace(0.5, 2.0, 23, device=dev)
        x, y = synth_images(B, 224, g, dev), torch.randint(0, 23, (B,), generator=g, device=dev)
        batch = (x, y)
        unl = B  # labeled images per step (the metric's unit for this workload)
        tfl = 3 * 2 * 1.8186e9 * B / 1e12  # resnet18 at 224^2: 1.8186 GMAC forward per image
        exe = tfl
        desc = (f"P0: supervised ResNet-18 step (timm resnet18, 23 classes; code/supervised.py:111-138), B={B}, "
                f"224^2, weighted CE, Adam 1e-3, EMA 0.999; convs with channels % 32 == 0 on bf16 MFMA "
                f"({'on' if model.conv_bf16 else 'off'}), the stem fp32; forward / backward "
                f"{'replayed as one hipGraph' if tr.use_graph else 'eager'}")
    else:
        from endossl.conformer import ConformerConfig, NativeConformer
        from endossl.semiformer import SemiFormer
        MU = 7
        if args.s1_model == "b384":
            # BASELINE configs[4] "ViT-Base/16 at 384^2": the reference's Conformer class defaults
            # (code/models/conformer.py:308-309: channel_ratio 4, embed_dim 768, depth 12, 12 heads) at
            # 384^2 (577 tokens), qkv_bias as build.py builds it.  Per GPU: B labeled + 2 mu B
            # unlabeled (B defaults to 8: ~0.75 GB of saved activations per image at this size)
            B = args.batch if args.batch != 64 else 8
            ccfg = ConformerConfig(img_size=384, channel_ratio=4, embed_dim=768, depth=12, heads=12)
            name = "Conformer-B (channel_ratio 4, embed 768, depth 12, 12 heads; code/models/conformer.py:308-309)"
        else:  # build.py's Conformer-Ti at 224^2, the B of kaggle_semisupervised_real_2.yaml:7
            B = args.batch if args.batch != 64 else 24
            ccfg = ConformerConfig()
            name = "Conformer-Ti (code/build.py:135-142: patch 16, embed 384, depth 12, 6 heads, channel_ratio 1)"
        S = ccfg.img_size
        model = NativeConformer(ccfg, seed=0)
        tr = SemiFormer(model, device=dev)
        cfg = AttrDict(DATA=AttrDict(BATCH_SIZE=B, MU=MU, IMG_SIZE=S, TARGET_NAME="target"),
                       MODEL=AttrDict(NAME="conformer", NUM_CLASSES=23),
                       TRAIN=AttrDict(IS_FREEZE=False, USE_EMA=True, EMA_DECAY=0.999, BASE_LR=1e-3, EVAL_STEP=1,
                                      EVAL_STEP_SUP=0, CLS_WEIGHT=False, THRES=0.95, T=1.0, LAMBDA_U=1.0, EPOCHS=1,
                                      WARMUP_EPOCHS=0, DECAY_EPOCHS=10, WARMUP_LR=5e-4, LR_DECAY=0.8, SCH_NAME="const"))
        tr.get_dataloader((None, None), None)
        tr.get_config(cfg)
        x, y = synth_images(B, S, g, dev), torch.randint(0, 23, (B,), generator=g, device=dev)
        batch = ((x, y), ((synth_images(B * MU, S, g, dev), synth_images(B * MU, S, g, dev)), None))
        unl, tfl = B * MU, conformer_step_tflop(ccfg, B + 2 * B * MU)
        exe = tfl
        desc = (f"S1: SemiFormer step on {name}, {S}^2 ({ccfg.T} tokens), B={B} + 2 x mu*B={B * MU} per GPU, C=23, "
                f"tau=0.95, lambda_u=1, EMA 0.999; transformer GEMMs and convs with channels % 32 == 0 on bf16 "
                f"MFMA ({'on' if model.conv_bf16 else 'off: ENDOSSL_CONV_BF16=0'}), CNN activation / gradient maps "
                f"{'bf16' if getattr(model, 'map_bf16', False) else 'fp32'}, BatchNorm statistics fp32")
        map_dtype = "bf16" if getattr(model, "map_bf16", False) else "fp32"
    steplog = args.steplog  # diagnostics: synchronises every step
    for _ in range(args.warmup):
        tr.step(batch)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        out = tr.step(batch)
        if steplog:
            torch.cuda.synchronize()
            print(f"step {i}: {1e3 * (time.perf_counter() - t0):.1f} ms cumulative, allocated "
                  f"{torch.cuda.memory_allocated(dev) / 2**30:.1f} GiB, reserved "
                  f"{torch.cuda.memory_reserved(dev) / 2**30:.1f} GiB, retries "
                  f"{torch.cuda.memory_stats(dev).get('num_alloc_retries', 0)}", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    dist.barrier()
    T = time.perf_counter() - t0
    elapsed = torch.tensor([T], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(elapsed, op=torch.distributed.ReduceOp.MAX)
    T = elapsed.item()
    host = None
    if args.host_input and args.workload in ("c1", "s1"):
        # C1 / S1 fed by the native host input path: TransformCoMatch's weak / strong_0 / strong_1 views
        # (C1) or TransformFixMatch's weak / strong pair (S1) and the labeled transform on the granted host
        # threads (csrc/host_aug.cpp), uint8 into the model (normalised on the device)
        import numpy as np

        from endossl import host_aug
        threads, _ = host_cpus()
        gh = np.random.default_rng(7)
        base = gh.integers(0, 256, (60, 80, 3), dtype=np.uint8)
        srcs = [host_aug.resize_bilinear(base ^ np.uint8(i * 29 % 256), (500, 375)) for i in range(64)]
        side = 224 if args.workload == "c1" else S
        lab = host_aug.HostBatcher(srcs, batch=B, size=side, kind="labeled", seed=1, threads=threads, device=dev)
        ub = host_aug.HostBatcher(srcs, batch=B * MU, size=side, kind="comatch" if args.workload == "c1" else "fixmatch",
                                  seed=2, threads=threads, device=dev)
        yh = torch.randint(0, 23, (B,), device=dev)

        def one():
            (xh,) = lab.next()
            return tr.step(((xh, yh), (ub.next(), None)))

        for _ in range(2):
            one()
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        for _ in range(args.steps):
            one()
        torch.cuda.synchronize()
        hd = time.perf_counter() - h0
        host = {"value": round(unl * args.steps / hd, 2), "unit": "unlabeled images/s",
                "ms_per_step": round(hd / args.steps * 1e3, 3), "host_threads": threads,
                "source": f"synthetic decoded RGB 500x375 frames (64), IS_CROP, S={side}; decode not timed"}
    if rank == 0:
        ms = T / args.steps * 1e3
        host_line = {"host_input": host} if host is not None else {}
        print(json.dumps({**{
            "metric": (f"labeled images/sec/node (P0)" if args.workload == "p0" else
                       f"unlabeled images/sec/node ({args.workload.upper()})"),
            "value": round(world * unl * args.steps / T, 2),
            "unit": "labeled images/s" if args.workload == "p0" else "unlabeled images/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": (f"bf16 operands (GEMMs, convs) / fp32 accumulate, BatchNorm statistics; CNN maps {map_dtype}"
                      if map_dtype else "bf16 operands (GEMMs, convs) / fp32 accumulate, maps, BatchNorm"),
            "data": "synthetic (HBM-resident, seed 0)", "config": {"workload": desc, "parallelism": f"dp{world}"},
            "step_tflop": round(tfl, 3), "executed_step_tflop": round(exe, 3),
            "step_tflops": round(tfl / (ms / 1e3), 1),
            # caching-allocator retries (a full cache flush + re-allocation each) slow a step by
            # orders of magnitude when HBM runs short: reported so such a run reads as one
            "hbm_peak_gib": round(torch.cuda.max_memory_allocated(dev) / 2**30, 1),
            "alloc_retries": int(torch.cuda.memory_stats(dev).get("num_alloc_retries", 0)),
            "device_allocs": int(torch.cuda.memory_stats(dev).get("num_device_alloc", 0)),
            "hbm_reserved_peak_gib": round(torch.cuda.max_memory_reserved(dev) / 2**30, 1),
            "final_loss": round(out["loss"].item(), 6)}, **host_line}), flush=True)
    dist.barrier()


def launcher_cmd(argv, nproc, port, script=None):
    """The torch.distributed.run command that runs this script once per GPU (one rank per GPU, RCCL
    over xGMI), with the same arguments, and the environment it needs."""
    script = script or os.path.abspath(__file__)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), script] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver (RCCL)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    return cmd, env


def _self_launch(args, argv):
    """`python bench.py --gpus N` (N > 1) with no WORLD_SIZE in the environment: start the N ranks as
    ONE child process (torch.distributed.run) before anything touches the GPU, let rank 0's JSON line
    pass through on the shared stdout, and exit with the child's status (no exec)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd, env = launcher_cmd(argv, args.gpus, port)
    print(f"bench.py: launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


def _check_world(args, world):
    if args.gpus != world:
        raise SystemExit(f"bench.py --gpus {args.gpus} but WORLD_SIZE={world}: launch N > 1 under "
                         f"`python -m torch.distributed.run --nproc-per-node {args.gpus} ... bench.py --gpus "
                         f"{args.gpus}` (one rank per GPU)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 200 timed steps by default (~6 s of GPU work at F1): long enough for an external utilisation sampler to
    # see the timed region, not only the CPU baseline
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="global labeled batch B (strong) / per-GPU B (weak)")
    ap.add_argument("--mu", type=int, default=7)
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=16, help="cpu_baseline labeled batch B (64 = the F1 batch)")
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--cpu-warmup", type=int, default=1)
    ap.add_argument("--inputs", choices=("u8", "f32"), default="u8",
                    help="F1 batch format in HBM: uint8 pixels (normalised in the patch gather) or fp32")
    ap.add_argument("--workload", choices=("f1", "c1", "s1", "p0"), default="f1",
                    help="f1 = the BASELINE metric (default); c1 / s1 = CoMatch / SemiFormer configs")
    ap.add_argument("--s1-model", choices=("b384", "ti224"), default="b384",
                    help="s1: the ViT-Base/16 384^2 stress Conformer (BASELINE configs[4]) or build.py's Conformer-Ti")
    ap.add_argument("--host-input", action="store_true",
                    help="also time F1 steps fed by the native host input path (endossl.host_aug.HostBatcher: "
                         "the reference's transforms on the granted host threads from decoded 500x375 RGB "
                         "frames, pinned uint8 batches copied on a side stream); reported as 'host_input', "
                         "never as value")
    ap.add_argument("--allreduce", choices=("auto", "single", "overlap"), default="auto",
                    help="N > 1: the gradient all-reduce as one launch after the backward (single), per-block "
                         "buckets overlapped with it (overlap), or auto = whichever ran faster in 3 untimed "
                         "steps each before the timed region (max over ranks)")
    ap.add_argument("--steplog", action="store_true", help="diagnostics: synchronise and log every timed step")
    ap.add_argument("--graph", choices=("auto", "on", "off"), default="auto",
                    help="hipGraph replay of the step's forward/backward (on); auto = off = eager launches "
                         "(measured faster than the replay at N = 1 and at the N = 8 shard, DESIGN.md §5)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_self_launch(args, sys.argv[1:]))
    if args.workload != "f1":
        return run_secondary(args)

    from endossl import dist
    from endossl.fixmatch import FixMatch
    from endossl.utils import AttrDict
    from endossl.vit import Engine, NativeViT, ViTConfig

    rank, world, local = dist.init_from_env()
    _check_world(args, world)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if args.scaling == "strong":
        if args.batch % world:
            raise SystemExit(f"strong scaling shards B={args.batch} over {world} ranks: B % N must be 0")
        B, MU = args.batch // world, args.mu  # this rank's shard: B/N labeled + mu*B/N pairs
    else:
        B, MU = args.batch, args.mu
    model = NativeViT(ViTConfig(), seed=0)
    tr = FixMatch(model, device=dev)
    # eager by default ("auto" = "off"): the captured-graph replay measured slower than eager launches
    # at both the per-rank shard of N = 8 (B = 8: 7.11 vs 6.40 ms/step) and the full batch (r02)
    graph = args.graph == "on"
    tr.use_graph = graph
    cfg = AttrDict(DATA=AttrDict(BATCH_SIZE=B, MU=MU, IMG_SIZE=224, TARGET_NAME="target"),
                   MODEL=AttrDict(NAME="vit_small_patch16_224", NUM_CLASSES=23),
                   TRAIN=AttrDict(IS_FREEZE=False, USE_EMA=True, EMA_DECAY=0.999, BASE_LR=1e-3, EVAL_STEP=1,
                                  CLS_WEIGHT=False, THRES=0.95, T=1.0, LAMBDA_U=1.0, EPOCHS=1, WARMUP_EPOCHS=0,
                                  DECAY_EPOCHS=10, WARMUP_LR=5e-4, LR_DECAY=0.8, SCH_NAME="const"))
    tr.get_dataloader((None, None), None)
    tr.get_config(cfg)
    # class weights as the SSL configs use (CLS_WEIGHT: True): balanced weights over 23 classes
    tr.class_weights = torch.linspace(0.5, 2.0, 23, device=dev)

    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    # default: the batch stays uint8 pixels in HBM and ToTensor + Normalize run inside the patch gather
    # (es_patch_im2col_u8, bit-identical patches); --inputs f32 hands over host-normalised fp32 images
    make = synth_u8 if args.inputs == "u8" else synth_images
    x = make(B, 224, g, dev)
    y = torch.randint(0, 23, (B,), generator=g, device=dev)
    uw = make(B * MU, 224, g, dev)
    us = make(B * MU, 224, g, dev)
    batch = ((x, y), ((uw, us), None))

    for _ in range(args.warmup):
        tr.step(batch)
    ar_probe = None
    if world > 1 and args.allreduce == "auto":
        # untimed: the gradient all-reduce as one launch after the backward vs per-block buckets overlapped
        # with it (FixMatch.overlap_allreduce), 3 steps each after 2 settling steps, max over ranks (so every
        # rank picks the same form); the timed steps run the faster one, the other is reported beside it
        ar_probe = {}
        for form in (False, True):
            tr.overlap_allreduce = form
            for _ in range(2):
                tr.step(batch)
            torch.cuda.synchronize()
            dist.barrier()
            p0 = time.perf_counter()
            for _ in range(3):
                tr.step(batch)
            torch.cuda.synchronize()
            dist.barrier()
            pe = torch.tensor([(time.perf_counter() - p0) / 3], dtype=torch.float64, device=dev)
            torch.distributed.all_reduce(pe, op=torch.distributed.ReduceOp.MAX)
            ar_probe["overlapped" if form else "single"] = round(pe.item() * 1e3, 3)
        tr.overlap_allreduce = ar_probe["overlapped"] < ar_probe["single"]
    elif world > 1:
        tr.overlap_allreduce = args.allreduce == "overlap"
    if graph and tr.static_batch() is not None:
        batch = tr.static_batch()  # the graph's own input buffers already hold this batch: no copy per step
    eng = model.engine()
    probe = {"label": "fc1_wgrad", "events": []}
    live = not graph  # HIP events bracket eager launches only
    if live:
        eng.probe = probe
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = tr.step(batch)
    torch.cuda.synchronize()
    dist.barrier()
    t1 = time.perf_counter()
    eng.probe = None
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(elapsed, op=torch.distributed.ReduceOp.MAX)
    T = elapsed.item()
    loss = out["loss"].item()

    # untimed steps after the timed region: the probed launch with the second stream off ("isolated"),
    # and, when the timed steps replayed a graph, the same launch co-scheduled as in the step
    use_graph, tr.use_graph = tr.use_graph, False
    if not live:
        eng.probe = probe
        for _ in range(2):
            tr.step(batch)
        torch.cuda.synchronize()
    ov = (eng.overlap, eng.overlap_fwd)
    eng.overlap = eng.overlap_fwd = False
    iso = {"label": "fc1_wgrad", "events": []}
    eng.probe = iso
    for _ in range(2):
        tr.step(batch)
    torch.cuda.synchronize()
    eng.probe = None
    eng.overlap, eng.overlap_fwd = ov
    tr.use_graph = use_graph
    weak = None
    if world > 1 and args.scaling == "strong":
        # configs[2] as the reference would run it under DDP: every rank a full B, mu batch (weak
        # scaling), timed the same way; reported beside the strong-scaling value (not the headline)
        xw, yw = make(args.batch, 224, g, dev), torch.randint(0, 23, (args.batch,), generator=g, device=dev)
        bw = ((xw, yw), ((make(args.batch * MU, 224, g, dev), make(args.batch * MU, 224, g, dev)), None))
        for _ in range(2):
            tr.step(bw)
        torch.cuda.synchronize()
        dist.barrier()
        w0 = time.perf_counter()
        for _ in range(args.steps):
            tr.step(bw)
        torch.cuda.synchronize()
        dist.barrier()
        we = torch.tensor([time.perf_counter() - w0], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(we, op=torch.distributed.ReduceOp.MAX)
        weak = {"per_gpu_batch": f"{args.batch} + {args.batch * MU} pairs",
                "value": round(world * args.batch * MU * args.steps / we.item(), 2),
                "ms_per_step": round(we.item() / args.steps * 1e3, 3),
                "note": "same step with every rank on a full B=64, mu=7 batch (DDP weak scaling)"}
        del xw, yw, bw
    ar_overlap = None
    if world > 1:
        # the same step with the OTHER all-reduce form (the headline runs the form --allreduce chose: with
        # `auto` the faster of the per-block buckets overlapped with the reverse pass -- FixMatch.
        # overlap_allreduce / dist.GradBuckets -- and one all-reduce after it), so one multi-GPU run measures both
        prev_ov, tr.overlap_allreduce = tr.overlap_allreduce, not tr.overlap_allreduce
        for _ in range(2):
            tr.step(batch)
        torch.cuda.synchronize()
        dist.barrier()
        a0 = time.perf_counter()
        for _ in range(args.steps):
            tr.step(batch)
        torch.cuda.synchronize()
        dist.barrier()
        ae = torch.tensor([time.perf_counter() - a0], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(ae, op=torch.distributed.ReduceOp.MAX)
        tr.overlap_allreduce = prev_ov
        ar_overlap = {"overlap_allreduce": not prev_ov, "value": round(world * B * MU * args.steps / ae.item(), 2),
                      "ms_per_step": round(ae.item() / args.steps * 1e3, 3),
                      "note": "same step and batch with the other all-reduce form (per-block buckets overlapped "
                              "with the backward vs one all-reduce after it)"}
    host_input = host_input_run(tr, B, MU, args.steps, dev) if args.host_input else None
    iso_ms = sum(e0.elapsed_time(e1) for e0, e1, _ in iso["events"]) / len(iso["events"])
    iso_tflops = (sum(f for _, _, f in iso["events"]) / (sum(e0.elapsed_time(e1) for e0, e1, _ in iso["events"]) / 1e3)
                  / 1e12)
    grouped = probe.get("kernel")  # the small-shard backward: the weight gradients as grouped launches
    layer = probe.get("layer_kernel")  # a block's weight gradients as one split-K launch (Engine.LAYER_WGRAD)
    ev_ms = [e0.elapsed_time(e1) for e0, e1, _ in probe["events"]]
    mean_ms = sum(ev_ms) / len(ev_ms)
    flop = sum(f for _, _, f in probe["events"]) / len(ev_ms)  # per launch (uniform at the fc1 site)
    tflops = sum(f for _, _, f in probe["events"]) / (sum(ev_ms) / 1e3) / 1e12
    M_tok = B * (1 + MU) * 197
    if layer:
        share = Engine.LAYER_TN_SHARE if ov[0] else 1.0
    else:
        share = (Engine.TN_SHARE if (ov[0] and not grouped and Engine.TN_SHARE < 1.0 and M_tok >= 16384) else 1.0)
    traffic, traffic_src = (None, None) if grouped else pmc_traffic("es_gemm_tn_big_grouped" if layer else "gemm_tn")
    lib = __import__("endossl._lib", fromlist=["load"]).load()
    tn_ws = lib.es_gemm_tn_workspace(1536, 384, 0)

    if rank == 0:
        ms = T / args.steps * 1e3
        glob_unl = world * B * MU  # unlabeled images the whole job processed per step
        work = STEP_TFLOP_F1 * glob_unl / 448.0
        res = {
            "metric": "unlabeled images/sec/node (FixMatch ViT-S, 224², μ=7)",
            "value": round(glob_unl * args.steps / T, 2),
            "unit": "unlabeled images/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
            "dtype": "bf16", "data": ("synthetic (HBM-resident uint8 pixels, ImageNet normalisation fused into the "
                                      "patch gather, seed 0)" if args.inputs == "u8" else
                                      "synthetic (HBM-resident uint8->ImageNet-normalised fp32, seed 0)"),
            "config": {"workload": f"F1: FixMatch ViT-S/16 step, global B={world * B} labeled + mu*B={glob_unl} "
                                   f"unlabeled weak/strong pairs ({B} + {B * MU} per GPU, {args.scaling} scaling), "
                                   f"224^2, C=23, tau=0.95, lambda_u=1, Adam 1e-3, EMA 0.999",
                       "global_batch": world * B * (1 + 2 * MU), "seq_len": 197, "parallelism": f"dp{world}",
                       "hipgraph": bool(graph)},
            "step_tflops": round(work / (ms / 1e3), 1),
            "step_mfma_frac": round(work / (ms / 1e3) / PEAK_BF16_TFLOPS / world, 4),
            "executed_step_tflop": round((STEP_TFLOP_F1 - (vit_s_pruned_tflop(448 + 512, 512)
                                                           if Engine.PRUNE_LAST else 0.0))
                                         * glob_unl / 448.0, 3),
            "final_loss": round(loss, 6),
            "roofline": {"kernel": (layer + " (bf16 operands, fp32 split-K slabs; rocprofv3: "
                                    "gemm_tn_big_grouped_kernel + splitk_reduce_grouped_kernel)" if layer else
                                    f"es_gemm_tn (weight gradient, fc1 site: out[1536, 384] = dY^T X over M={M_tok} "
                                    "train tokens, bf16 operands, fp32 split-K slabs + reduction, fused bias "
                                    "gradient); rocprofv3: gemm_tn_big_kernel + splitk_reduce_kernel"
                                    if not grouped else
                                    f"{grouped}: every weight gradient of the backward over M={M_tok} train tokens "
                                    "(Engine.GROUP_WGRAD, small shard), one launch per 4 layers, bf16 operands, "
                                    "whole-axis 128x128 tiles, fused bias gradients; rocprofv3: "
                                    "gemm_tn_grouped_kernel"),
                         "bound": "mfma", "achieved": round(tflops, 1), "peak": round(PEAK_BF16_TFLOPS, 1),
                         "unit": "TFLOP/s", "frac": round(tflops / PEAK_BF16_TFLOPS, 4), "traffic": traffic,
                         "traffic_source": (traffic_src + " (a separate rocprofv3 --pmc pass over this bench, "
                                            "not measured in this run)") if traffic_src else None,
                         "algorithmic_flop": flop, "mean_launch_ms": round(mean_ms, 4), "launches": len(ev_ms),
                         "algorithmic_bytes": probe.get("layer_bytes"),
                         "timed": ("live in the timed steps" if live else "2 untimed eager steps after the timed "
                                                                          "(graph-replayed) steps")
                                  + ("; by events the kernel dispatches stamp themselves (hipExtLaunchKernelGGL: "
                                     "from the grouped kernel's start to the reduce launch's end, the span a "
                                     "rocprofv3 kernel trace shows, not the stream position of an event record)"
                                     if layer else ""),
                         "streams": 2 if ov[0] else 1, "tn_workspace_floats": int(tn_ws),
                         "cu_share": share,
                         "frac_of_share": round(tflops / (PEAK_BF16_TFLOPS * share), 4),
                         "share_note": ("the live launch is sized to this share of the CUs (Engine.TN_SHARE: "
                                        "the rest run the data-gradient chain beside it); frac is against the "
                                        "whole chip's peak, frac_of_share against the granted CUs' peak"),
                         "isolated": {"mean_launch_ms": round(iso_ms, 4),
                                      "achieved": round(iso_tflops, 1),
                                      "frac": round(iso_tflops / PEAK_BF16_TFLOPS, 4),
                                      "note": "same launch with the engine's second HIP stream off (2 untimed "
                                              "steps): the live figure shares the CUs with the data-gradient chain"}},
        }
        sc, sc_src = step_counters()
        if sc is not None and world == 1:
            busy = sc["step"]["mfma_busy_simd_cycles"]
            same = sc.get("lib_sha256") is not None and sc.get("lib_sha256") == lib_sha256()
            res["mfma_util"] = {
                "value": round(busy / (1024 * (ms / 1e3) * 2.4e9), 4),
                "kind": ("counters measured on this library build" if same else
                         "ESTIMATE: counters measured on another library build (" + str(sc.get("lib_sha256"))[:16] + ")"),
                "mfma_busy_simd_cycles_per_step": busy,
                "profiled": {k: round(v, 4) for k, v in sc["step"].items() if k.startswith(("mfma_util", "effective"))},
                "hbm_bytes_per_step": sc["step"]["hbm_bytes"],
                "hbm_tbs_at_this_step_time": round(sc["step"]["hbm_bytes"] / (ms / 1e3) / 1e12, 3),
                "source": (sc_src + " (rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES / FETCH_SIZE / WRITE_SIZE passes over "
                           "this bench; committed, not measured in this run)"),
                "note": "value = the step's MFMA-busy SIMD-cycles / (1024 SIMDs x this run's ms_per_step x 2.4 GHz "
                        "nominal): a lower bound (the chip holds a lower clock under load); per-family figures in "
                        "the .md"}
        if weak is not None:
            res["weak_scaling"] = weak
        if ar_overlap is not None:
            res["allreduce_form"] = "overlapped per-block buckets" if tr.overlap_allreduce else "one after the backward"
            res["allreduce_other_form"] = ar_overlap
            if ar_probe is not None:
                res["allreduce_choice"] = {"probe_ms_per_step": ar_probe,
                                           "note": "--allreduce auto: both forms timed for 3 untimed steps before the "
                                                   "timed region (max over ranks); the faster one is the headline"}
        if host_input is not None:
            res["host_input"] = host_input
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(B=args.cpu_batch, steps=args.cpu_steps, warmup=args.cpu_warmup)
        print(json.dumps(res), flush=True)
    dist.barrier()


if __name__ == "__main__":
    main()

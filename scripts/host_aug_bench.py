"""Host input-path throughput: TransformFixMatch (weak + strong) and the labeled transform on the
native library (csrc/host_aug.cpp) vs PIL doing the same ops in-process, per host thread count.
Source images: synthetic RGB 500 x 375 (a typical endoscopy frame aspect), IS_CROP, S = 224.

  python scripts/host_aug_bench.py [--n 256] [--threads 1,4,16]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
import numpy as np  # noqa: E402

from endossl import host_aug  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--threads", default="1,4,16")
    ap.add_argument("--size", type=int, default=224)
    args = ap.parse_args()
    g = np.random.default_rng(0)
    base = g.integers(0, 256, (47, 63, 3), dtype=np.uint8)
    imgs = [host_aug.resize_bilinear(base + np.uint8(i % 7), (500, 375)) for i in range(args.n)]
    res = {"n": args.n, "size": args.size, "src": "500x375", "cpus": os.cpu_count()}
    for t in [int(x) for x in args.threads.split(",")]:
        host_aug.transform_batch(imgs[:8], args.size, "fixmatch", threads=t)
        t0 = time.perf_counter()
        host_aug.transform_batch(imgs, args.size, "fixmatch", seed=1, threads=t)
        dt = time.perf_counter() - t0
        t1 = time.perf_counter()
        host_aug.transform_batch(imgs, args.size, "labeled", seed=1, threads=t)
        dl = time.perf_counter() - t1
        res[f"threads{t}"] = {"fixmatch_pairs_per_s": round(args.n / dt, 1), "labeled_per_s": round(args.n / dl, 1)}
    try:  # the same weak + strong ops through PIL, one thread (what a DataLoader worker runs)
        from PIL import Image, ImageOps
        k = min(args.n, 64)
        t0 = time.perf_counter()
        for a in imgs[:k]:
            im = Image.fromarray(a).resize((int(args.size * 1.2),) * 2, Image.BILINEAR)
            off = (im.size[0] - args.size) // 2
            im = im.crop((off, off, off + args.size, off + args.size))
            np.asarray(im)
            s = ImageOps.mirror(im).rotate(13)
            s = ImageOps.equalize(s)
            np.asarray(s)
        res["pil_1thread_pairs_per_s_approx"] = round(k / (time.perf_counter() - t0), 1)
    except ImportError:
        pass
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

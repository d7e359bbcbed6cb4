"""Generate the committed golden fixtures from the CPU oracle (test infrastructure).

  golden_small.npz   full input and output buffers of a 1,000-Gaussian 64x64 scene
  golden_cfg1.npz    config 1 (10k Gaussians, 256x256, seed 1): inputs + SHA-256 of every
                     integer/byte output, float colours and per-field gradient sums/norms

The reference itself cannot run in this image (Objective-C++/Metal), so these vectors pin the
oracle (the CPU restatement, cross-checked by tests/kat_reference.py), not the reference binary:
"parity unpinned" (DESIGN.md §4). Run: python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from gaussiansplatting_amd import scene  # noqa: E402
from oracle import oracle  # noqa: E402


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def run(n, w, h, seed):
    g = scene.synthetic_gaussians(n, seed, w, h)
    u = scene.make_uniforms(w, h)
    gt = scene.synthetic_ground_truth(seed, 0, w, h)
    f = oracle.forward(g, u, w, h, threads=1)
    gr, ab, nz = oracle.backward(g, f, f.rgba8, gt, threads=1)
    return g, u, gt, f, gr, ab, nz


def main():
    live = [o for _, o in scene.GRAD_FIELDS]
    g, u, gt, f, gr, ab, nz = run(1000, 64, 64, 42)
    np.savez_compressed(os.path.join(HERE, "golden_small.npz"), gaussians=g, uniforms=u, gt=gt,
                        keys=f.keys, values=f.values, ranges=f.ranges, last_idx=f.last_idx,
                        rgba8=f.rgba8, rgb=f.rgb, projected=f.projected, grad=gr[:, live],
                        grad_abs=ab[:, live], grad_noise=nz[:, live])
    c = scene.CONFIGS[1]
    g, u, gt, f, gr, ab, nz = run(c["n"], c["width"], c["height"], c["seed"])
    np.savez_compressed(
        os.path.join(HERE, "golden_cfg1.npz"), gaussians=g, uniforms=u, gt=gt,
        num_pairs=np.uint64(f.num_pairs),
        sha_keys=sha(f.keys), sha_values=sha(f.values), sha_ranges=sha(f.ranges),
        sha_last_idx=sha(f.last_idx), sha_rgba8=sha(f.rgba8), sha_rgb=sha(f.rgb),
        sha_projected=sha(f.projected),
        grad_sum=gr[:, live].sum(0), grad_abs_sum=np.abs(gr[:, live]).sum(0),
        grad_norm=np.sqrt((gr[:, live] ** 2).sum(0)))
    print("P small", len(np.load(os.path.join(HERE, "golden_small.npz"))["keys"]), "P cfg1", f.num_pairs)


if __name__ == "__main__":
    main()

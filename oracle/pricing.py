"""IR comparison of two oracle arithmetics on the same rays (test infrastructure, like the oracle).

Used by tests/test_oracle_reference_arith.py and tools/arith_pricing.py: per-ray final records
(orc_trace_records) traced on a thread pool, the two ears' IRs rebuilt from them the way
devicePrograms.cu:128-170 adds a receiver hit, and the metrics of DESIGN.md section 3: every ray
classed as identical / same path with a bin flip / diverged, each class's share of the per-bin
relative RMS, the bin-tolerant RMS of the same-path rays (the arithmetic), the 1-ms energy curve,
Schroeder's energy decay curve.
"""
from __future__ import annotations

import concurrent.futures as cf
import ctypes as C
import os

import numpy as np

import pyoracle as po

REC = np.dtype([("energy", np.float32), ("distance", np.float32), ("depth", np.int32), ("bin", np.int32),
                ("queries", np.int32), ("last_tri", np.int32), ("path_hash", np.uint32)])


def records(osc: po.Scene, p, begin: int, end: int, threads: int | None = None, chunk: int = 20000) -> np.ndarray:
    """orc_trace_records over rays [begin, end), chunked over a thread pool (ctypes drops the GIL)."""
    out = np.empty(end - begin, REC)
    assert REC.itemsize == C.sizeof(po.OrcRayRecord)

    def run(b):
        n = min(chunk, end - b)
        view = out[b - begin:b - begin + n]
        po.lib().orc_trace_records(C.byref(osc.s), C.byref(p), b, n,
                                   C.cast(view.ctypes.data, C.POINTER(po.OrcRayRecord)))

    with cf.ThreadPoolExecutor(threads or os.cpu_count() or 8) as ex:
        list(ex.map(run, range(begin, end, chunk)))
    return out


def ir_from_records(rec: np.ndarray, ta: np.ndarray, ir_len: int, sr: int, hrtf: float, mask=None):
    """The two ears' IRs (f64 sums of the f32 contributions) of the rays whose last query hit a
    receiver half: the own ear gets e at bin k, the other e * (1 - hrtf) at k + delay (or k past the
    end), devicePrograms.cu:125-170."""
    delay = int(sr * 0.00044)
    hit = (rec["depth"] == -1) & (rec["last_tri"] >= 0) & (rec["bin"] >= 0) & (rec["bin"] < ir_len)
    hit &= ta[np.maximum(rec["last_tri"], 0)] < 0
    if mask is not None:
        hit &= mask
    r = rec[hit]
    left = ta[r["last_tri"]] == -1.0
    k = r["bin"].astype(np.int64)
    kk = np.where(k + delay < ir_len, k + delay, k)
    e = r["energy"].astype(np.float32)
    ec = (e * np.float32(1.0 - hrtf)).astype(np.float32)
    L = np.zeros(ir_len)
    R = np.zeros(ir_len)
    np.add.at(L, k[left], e[left])
    np.add.at(R, kk[left], ec[left])
    np.add.at(R, k[~left], e[~left])
    np.add.at(L, kk[~left], ec[~left])
    return L, R


def rel_rms(a, b) -> float:
    n = np.linalg.norm(a)
    return float(np.linalg.norm(a - b) / n) if n else 0.0


def energy_curve(ir, sr, ms=1.0):
    """Energy per `ms` window: the IR as an energy-time curve."""
    w = max(1, int(sr * ms / 1000))
    n = len(ir) // w * w
    return ir[:n].reshape(-1, w).sum(1)


def edc(ir):
    """Schroeder's energy decay curve: the energy still to arrive after each bin."""
    return np.cumsum(ir[::-1])[::-1]


def bin_position(rec: np.ndarray, sr: int, arith: int) -> np.ndarray:
    """The real-valued bin k = (dist / 343) * sr before rounding, computed as each arithmetic does
    (devicePrograms.cu:131-132): IEEE f32 division (arith 0 / 2) or div.approx modelled as
    dist * rcp(343) (arith 1, arx_oracle.c rf_div)."""
    d = rec["distance"].astype(np.float32)
    if arith == 1:
        q = (d * np.float32(1.0 / 343.0)).astype(np.float32)
    else:
        q = (d / np.float32(343.0)).astype(np.float32)
    return (q * np.float32(sr)).astype(np.float32)


def _is_receiver(rec, ta, ir_len):
    return (rec["depth"] == -1) & (rec["last_tri"] >= 0) & (rec["bin"] >= 0) & (rec["bin"] < ir_len) & \
        (ta[np.maximum(rec["last_tri"], 0)] < 0)


def compare(a: np.ndarray, b: np.ndarray, ta, ir_len: int, sr: int, hrtf: float, arith_a: int = 0,
            arith_b: int = 1) -> dict:
    """Metrics of IR b against IR a (a's norm in the denominators), both from per-ray records of the
    same ray ids, with every ray in one of three classes:
      identical  the same path (the same closest-hit triangle sequence, path_hash, and the same query
                 count) and the same bin -- only the energy's arithmetic differs;
      bin flip   the same path, another bin: roundf((dist / 343) * sr) (devicePrograms.cu:131-132) on
                 the two sides of a .5 boundary, dist (:83) differing by ulps;
      diverged   another path: a query met a triangle edge within an ulp and hit another triangle.
    Each class's contribution is the relative RMS of IR a against the IR of a's records with that
    class's rays taken from b.  "tolerant" metrics let a same-path receiver hit land within one bin of
    a's (its energy is compared in a's bin): the arithmetic's energy error with the bin flips counted."""
    same_path = (a["last_tri"] == b["last_tri"]) & (a["queries"] == b["queries"]) & (a["path_hash"] == b["path_hash"])
    same_bin = a["bin"] == b["bin"]
    identical = same_path & same_bin
    flip = same_path & ~same_bin
    diverged = ~same_path
    ra, rb = _is_receiver(a, ta, ir_len), _is_receiver(b, ta, ir_len)

    def ir(rec, mask=None):
        return ir_from_records(rec, ta, ir_len, sr, hrtf, mask)

    def mix(mask):  # a's records with the class's rays taken from b
        m = a.copy()
        m[mask] = b[mask]
        return m

    b_tol = b.copy()  # same-path hits within one bin compared in a's bin
    tol = flip & (np.abs(a["bin"].astype(np.int64) - b["bin"]) <= 1)
    b_tol["bin"][tol] = a["bin"][tol]
    La, Ra = ir(a)
    Lb, Rb = ir(b)
    Las, Ras = ir(a, same_path)
    Lbs, Rbs = ir(b, same_path)
    Lbt, Rbt = ir(b_tol, same_path)
    Lat, Rat = ir(b_tol)
    contrib = {}
    for name, mask in (("identical", identical), ("bin_flip", flip), ("diverged", diverged)):
        Lm, Rm = ir(mix(mask))
        contrib[name] = {"L": rel_rms(La, Lm), "R": rel_rms(Ra, Rm)}
    # the bin flips against the rounding they come from: both sides' real-valued bins x, their
    # distance |x_a - x_b| in bins, and the count a uniform fractional position predicts (sum |dx|)
    rf = same_path & ra & rb
    xa, xb = bin_position(a[rf], sr, arith_a), bin_position(b[rf], sr, arith_b)
    dx = np.abs(xa.astype(np.float64) - xb.astype(np.float64))
    fl = flip[rf]
    queries = int(a["queries"].sum())
    return {
        "rel_rms_L": rel_rms(La, Lb), "rel_rms_R": rel_rms(Ra, Rb),
        "rel_rms_same_path_L": rel_rms(Las, Lbs), "rel_rms_same_path_R": rel_rms(Ras, Rbs),
        "rel_rms_same_path_tolerant_L": rel_rms(Las, Lbt), "rel_rms_same_path_tolerant_R": rel_rms(Ras, Rbt),
        "rel_rms_tolerant_L": rel_rms(La, Lat), "rel_rms_tolerant_R": rel_rms(Ra, Rat),
        "rel_rms_1ms_energy_L": rel_rms(energy_curve(La, sr), energy_curve(Lb, sr)),
        "rel_rms_1ms_energy_R": rel_rms(energy_curve(Ra, sr), energy_curve(Rb, sr)),
        "rel_rms_edc_L": rel_rms(edc(La), edc(Lb)), "rel_rms_edc_R": rel_rms(edc(Ra), edc(Rb)),
        "contribution": contrib,
        "rays": int(len(a)),
        "rays_identical": int(identical.sum()),
        "rays_bin_flip": int(flip.sum()),
        "rays_other_path": int(diverged.sum()),
        "other_path_per_query": float(diverged.sum() / max(1, queries)),
        "receiver_rays_bin_flip": int((flip & (ra | rb)).sum()),
        "receiver_rays_other_path": int((diverged & (ra | rb)).sum()),
        "receiver_rays_other_bin": int(((ra | rb) & ~same_bin).sum()),
        "receiver_rays": int(ra.sum()),
        "bin_flip_max_step": int(np.abs(a["bin"][flip].astype(np.int64) - b["bin"][flip]).max()) if flip.any() else 0,
        "bin_flip_max_dx": float(dx[fl].max()) if fl.any() else 0.0,
        "bin_flip_predicted": float(dx.sum()),
        "same_path_receiver_max_dx": float(dx.max()) if dx.size else 0.0,
        "same_path_receiver_rays": int(rf.sum()),
        "queries": [queries, int(b["queries"].sum())],
    }


# the bars the build's IEEE convention meets against the reference's compiled
# arithmetic on the same rays (round 5: the three ray classes of compare()).
#   arith_tolerant_rel_rms  per-bin relative RMS over the same-path rays, a hit allowed to land one bin
#                           off (the bin flips counted, their energy compared in a's bin): the arithmetic;
#   bin_flips_rounding      every same-path bin change is one bin, no same-path receiver ray's real-valued
#                           bin drifts by BIN_FLIP_DX or more between the arithmetics (its dist differs by
#                           ulps summed over its segments, not by a path), and the flip count is what
#                           rounding at that drift predicts (sum |x_a - x_b|, Poisson bounds);
#   edc_rel_rms             Schroeder's decay curve (the integral RT60 and clarity are read from);
#   energy_1ms_rel_rms      the 1-ms energy-time curve, every ray and every flip counted;
#   other_path_per_query    rays whose path diverges (an edge hit one ulp apart) per closest-hit query --
#                           any triangle of the sequence (path_hash), so also paths that rejoin: <= 3e-4,
#                           and no more than 1.1x the IEEE arithmetic with the reference's own reflection
#                           formula (arith 2) diverges from the reference arithmetic;
#   diverged_rel_rms        per-bin relative RMS the diverged rays contribute;
#   per_bin_vs_seed_spread  per-bin relative RMS over the reference's own Monte-Carlo spread (two seeds
#                           = two runs of the clock64-seeded launch, devicePrograms.cu:216-217), bounded
#                           by what re-drawing the diverged and flipped rays could cause.
BARS = {"arith_tolerant_rel_rms": 1e-4, "edc_rel_rms": 1e-4, "energy_1ms_rel_rms": 2e-3,
        "other_path_per_query": 3e-4, "diverged_rel_rms": 2e-3}
BIN_FLIP_DX = 0.25  # bins (1.8 mm of path at 48 kHz)
OTHER_PATH_VS_REFERENCE_FORM = 1.1


def _worse(m: dict, key: str) -> float:
    return max(m[key + "_L"], m[key + "_R"])


def bin_flips_explained(m: dict) -> tuple[bool, dict]:
    pred = m["bin_flip_predicted"]
    n = m["receiver_rays_bin_flip"]
    lo, hi = pred - 4.0 * np.sqrt(pred) - 3.0, pred + 4.0 * np.sqrt(pred) + 3.0
    ok = (m["bin_flip_max_step"] <= 1) and (m["same_path_receiver_max_dx"] < BIN_FLIP_DX) and (lo <= n <= hi)
    return bool(ok), {"flips": n, "predicted": pred, "bounds": [lo, hi], "max_step": m["bin_flip_max_step"],
                      "max_dx_flips": m["bin_flip_max_dx"], "max_dx_same_path": m["same_path_receiver_max_dx"],
                      "dx_bar": BIN_FLIP_DX}


def bars_met(ieee_vs_ref: dict, seed_spread: dict, reference_form: dict | None = None) -> dict:
    """Each bar's measured value (the worse ear) and whether it holds; reference_form = compare() of
    the IEEE arithmetic with the reference's normalize(cr) reflection (arith 2) against the reference
    arithmetic, for the relative divergence bar."""
    m = ieee_vs_ref
    vals = {
        "arith_tolerant_rel_rms": _worse(m, "rel_rms_same_path_tolerant"),
        "edc_rel_rms": _worse(m, "rel_rms_edc"),
        "energy_1ms_rel_rms": _worse(m, "rel_rms_1ms_energy"),
        "other_path_per_query": m["other_path_per_query"],
        "diverged_rel_rms": max(m["contribution"]["diverged"]["L"], m["contribution"]["diverged"]["R"]),
        "per_bin_vs_seed_spread": max(m["rel_rms_L"] / max(seed_spread["rel_rms_L"], 1e-30),
                                      m["rel_rms_R"] / max(seed_spread["rel_rms_R"], 1e-30)),
    }
    redraw = float(np.sqrt((m["rays_other_path"] + m["rays_bin_flip"]) / max(1, m["rays"])))
    bars = dict(BARS, per_bin_vs_seed_spread=redraw + 1e-4)
    out = {k: {"value": v, "bar": bars[k], "ok": bool(v <= bars[k])} for k, v in vals.items()}
    ok, detail = bin_flips_explained(m)
    out["bin_flips_rounding"] = dict(detail, ok=ok)
    if reference_form is not None:
        v = m["other_path_per_query"] / max(reference_form["other_path_per_query"], 1e-30)
        out["other_path_vs_reference_form"] = {"value": v, "bar": OTHER_PATH_VS_REFERENCE_FORM,
                                               "ok": bool(v <= OTHER_PATH_VS_REFERENCE_FORM)}
    return out

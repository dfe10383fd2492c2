"""IR comparison of two oracle arithmetics on the same rays (test infrastructure, like the oracle).

Used by tests/test_oracle_reference_arith.py and tools/arith_pricing.py: per-ray final records
(orc_trace_records) traced on a thread pool, the two ears' IRs rebuilt from them the way
devicePrograms.cu:128-170 adds a receiver hit, and the metrics of DESIGN.md section 3 -- per-bin
relative RMS, the same over the rays whose path agrees, the 1-ms energy curve, Schroeder's energy
decay curve, and how many rays take another path.
"""
from __future__ import annotations

import concurrent.futures as cf
import ctypes as C
import os

import numpy as np

import pyoracle as po

REC = np.dtype([("energy", np.float32), ("distance", np.float32), ("depth", np.int32), ("bin", np.int32),
                ("queries", np.int32), ("last_tri", np.int32)])


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


def compare(a: np.ndarray, b: np.ndarray, ta, ir_len: int, sr: int, hrtf: float) -> dict:
    """Metrics of IR b against IR a (a's norm in the denominators), both from per-ray records of the
    same ray ids.  A ray "takes another path" when its last triangle, its query count or its bin
    differ."""
    same = (a["last_tri"] == b["last_tri"]) & (a["queries"] == b["queries"]) & (a["bin"] == b["bin"])
    recv_a = (a["bin"] >= 0) & (a["bin"] < ir_len)
    recv_b = (b["bin"] >= 0) & (b["bin"] < ir_len)
    La, Ra = ir_from_records(a, ta, ir_len, sr, hrtf)
    Lb, Rb = ir_from_records(b, ta, ir_len, sr, hrtf)
    Las, Ras = ir_from_records(a, ta, ir_len, sr, hrtf, same)
    Lbs, Rbs = ir_from_records(b, ta, ir_len, sr, hrtf, same)
    queries = int(a["queries"].sum())
    return {
        "rel_rms_L": rel_rms(La, Lb), "rel_rms_R": rel_rms(Ra, Rb),
        "rel_rms_same_path_L": rel_rms(Las, Lbs), "rel_rms_same_path_R": rel_rms(Ras, Rbs),
        "rel_rms_1ms_energy_L": rel_rms(energy_curve(La, sr), energy_curve(Lb, sr)),
        "rel_rms_1ms_energy_R": rel_rms(energy_curve(Ra, sr), energy_curve(Rb, sr)),
        "rel_rms_edc_L": rel_rms(edc(La), edc(Lb)), "rel_rms_edc_R": rel_rms(edc(Ra), edc(Rb)),
        "rays": int(len(a)),
        "rays_other_path": int((~same).sum()),
        "other_path_per_query": float((~same).sum() / max(1, queries)),
        "receiver_rays_other_bin": int(((recv_a | recv_b) & (a["bin"] != b["bin"])).sum()),
        "receiver_rays": int(recv_a.sum()),
        "queries": [queries, int(b["queries"].sum())],
    }


# the bars the build's IEEE convention meets against the reference's compiled
# arithmetic on the same rays.
#   same_path_rel_rms     per-bin relative RMS over the rays whose path agrees: the arithmetic itself;
#   edc_rel_rms           Schroeder's decay curve (the integral RT60 and clarity are read from);
#   other_path_per_query  rays whose path diverges (an edge hit one ulp apart) per closest-hit query;
#   per_bin_vs_seed_spread  per-bin relative RMS over the reference's own Monte-Carlo spread (two seeds
#                         = two runs of the clock64-seeded launch, devicePrograms.cu:216-217), bounded
#                         by what re-drawing the diverged rays could cause: sqrt(diverged / rays)
#                         (+ 1e-4 for the arithmetic of the rest).
BARS = {"same_path_rel_rms": 1e-4, "edc_rel_rms": 1e-4, "other_path_per_query": 2e-4}


def bars_met(ieee_vs_ref: dict, seed_spread: dict) -> dict:
    """Each bar's measured value (the worse ear) and whether it holds."""
    m = {
        "same_path_rel_rms": max(ieee_vs_ref["rel_rms_same_path_L"], ieee_vs_ref["rel_rms_same_path_R"]),
        "edc_rel_rms": max(ieee_vs_ref["rel_rms_edc_L"], ieee_vs_ref["rel_rms_edc_R"]),
        "other_path_per_query": ieee_vs_ref["other_path_per_query"],
        "per_bin_vs_seed_spread": max(ieee_vs_ref["rel_rms_L"] / max(seed_spread["rel_rms_L"], 1e-30),
                                      ieee_vs_ref["rel_rms_R"] / max(seed_spread["rel_rms_R"], 1e-30)),
    }
    redraw = float(np.sqrt(ieee_vs_ref["rays_other_path"] / max(1, ieee_vs_ref["rays"])))
    bars = dict(BARS, per_bin_vs_seed_spread=redraw + 1e-4)
    return {k: {"value": v, "bar": bars[k], "ok": bool(v <= bars[k])} for k, v in m.items()}

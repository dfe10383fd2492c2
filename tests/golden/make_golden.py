#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ (run in the build container only).

Inputs come from the reference checkout (/root/reference, read-only) through
oracle/_ref/refdump -- a driver linking the reference's own tinyobj v2.0.0,
AudioFile.h, cJSON and glm, compiled from the reference tree by
`make -C oracle ref`.  Fixtures are DATA: loader outputs (triangulated meshes,
decoded samples) and parsed config values.  Nothing here is copied source.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("ARX_REFERENCE", "/root/reference")
REFDUMP = os.path.join(REPO, "oracle", "_ref", "refdump")
MODELS = os.path.join(REF, "assets", "models")


def refdump(*args: str) -> list[str]:
    out = subprocess.run([REFDUMP, *args], check=True, capture_output=True, text=True).stdout
    return out.splitlines()


def parse_meshes(lines: list[str]) -> dict:
    i = 0
    header = {}
    if lines[0].startswith("shapes"):
        tok = lines[0].split()
        header = {"shapes": int(tok[1]), "materials": int(tok[3]), "vertices": int(tok[5])}
        i = 1
    assert lines[i].startswith("meshes")
    n = int(lines[i].split()[1])
    i += 1
    names, verts, idxs = [], [], []
    for _ in range(n):
        _, name, nv, nt = lines[i].split()
        nv, nt = int(nv), int(nt)
        i += 1
        v = np.array([float.fromhex(x) for x in lines[i:i + 3 * nv]], dtype=np.float32).reshape(nv, 3)
        i += 3 * nv
        f = np.array([int(x) for x in lines[i:i + 3 * nt]], dtype=np.int32).reshape(nt, 3)
        i += 3 * nt
        names.append(name)
        verts.append(v)
        idxs.append(f)
    return {"header": header, "names": names, "vertices": verts, "indices": idxs}


def save_meshes(path: str, m: dict) -> None:
    arrays = {"names": np.array(m["names"])}
    for k, (v, f) in enumerate(zip(m["vertices"], m["indices"])):
        arrays[f"v{k}"] = v
        arrays[f"f{k}"] = f
    if m["header"]:
        arrays["header"] = np.array([m["header"]["shapes"], m["header"]["materials"], m["header"]["vertices"]])
    np.savez_compressed(path, **arrays)


def wav_fixture(path: str) -> dict:
    lines = refdump("wav", path)
    sr, ch, n, bits = (int(x) for x in lines[0].split()[1:])
    data = np.array([float.fromhex(x) for x in lines[1:]], dtype=np.float32).reshape(ch, n)
    return {
        "file": os.path.relpath(path, REF),
        "sample_rate": sr, "channels": ch, "samples_per_channel": n, "bit_depth": bits,
        "head": [[float(x) for x in data[c, :256]] for c in range(ch)],
        "strided_997": [[float(x) for x in data[c, ::997]] for c in range(ch)],
        "sum": [float(np.sum(data[c], dtype=np.float64)) for c in range(ch)],
        "sumsq": [float(np.sum(data[c].astype(np.float64) ** 2)) for c in range(ch)],
    }


def audio_fixture(path: str, out: str) -> None:
    """Channel 0 of a reference WAV as the reference's AudioFile decoded it, for the GPU tests and
    bench.py (the reference tree is absent on the GPU box).  16-bit PCM is stored as its integer
    codes (AudioFile: sample = code / 32768, AudioFile.h:1242-1245), IEEE float as float32."""
    lines = refdump("wav", path)
    sr, ch, n, bits = (int(x) for x in lines[0].split()[1:])
    x = np.array([float.fromhex(v) for v in lines[1:1 + n]], dtype=np.float32)
    if bits == 16:
        codes = np.rint(x.astype(np.float64) * 32768.0).astype(np.int16)
        assert np.array_equal((codes.astype(np.float32) / np.float32(32768.0)), x)
        np.savez_compressed(out, sample_rate=sr, bit_depth=bits, channels=ch, pcm16=codes)
    else:
        np.savez_compressed(out, sample_rate=sr, bit_depth=bits, channels=ch, f32=x)


def audio_fixtures() -> None:
    audio_fixture(os.path.join(REF, "guitar_sample_16k.wav"), os.path.join(HERE, "audio_guitar_16k_ch0.npz"))
    audio_fixture(os.path.join(REF, "experimento_entrada_16KHz.wav"), os.path.join(HERE, "audio_experimento_16k_ch0.npz"))
    audio_fixture(os.path.join(REF, "assets", "sound_samples", "A_Clapper_Board.wav"),
                  os.path.join(HERE, "audio_clapper_48k_ch0.npz"))


def main() -> int:
    if len(sys.argv) > 1 and sys.argv[1] == "audio":
        audio_fixtures()
        return 0
    if not os.path.exists(REFDUMP):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    left = os.path.join(MODELS, "leftHalf.obj")
    right = os.path.join(MODELS, "rightHalf.obj")
    # receiver halves in their local frame (placement (0,0,0), yaw 0 -> glm identity)
    save_meshes(os.path.join(HERE, "receiver_local.npz"), parse_meshes(refdump("receiver", left, right, "0", "0", "0", "0")))
    # C1 placement (R/config.json initial_receiver_pos, yaw 0) and a rotated one
    save_meshes(os.path.join(HERE, "receiver_c1.npz"), parse_meshes(refdump("receiver", left, right, "2.5", "9.9", "0", "0")))
    save_meshes(os.path.join(HERE, "receiver_rot.npz"), parse_meshes(refdump("receiver", left, right, "-1.25", "2.0", "3.5", "37.5")))
    for name in ("test", ):
        save_meshes(os.path.join(HERE, f"{name}_obj.npz"), parse_meshes(refdump("obj", os.path.join(REF, f"{name}.obj"))))
    for name in ("3D_U", "cajaConToro", "planaso2"):
        save_meshes(os.path.join(HERE, f"{name}_obj.npz"), parse_meshes(refdump("obj", os.path.join(MODELS, f"{name}.obj"))))
    wavs = [wav_fixture(os.path.join(REF, "guitar_sample_16k.wav")),
            wav_fixture(os.path.join(REF, "experimento_entrada_16KHz.wav")),
            wav_fixture(os.path.join(REF, "assets", "sound_samples", "A_Clapper_Board.wav"))]
    with open(os.path.join(HERE, "wav_decode.json"), "w") as fh:
        json.dump(wavs, fh)
    audio_fixtures()
    cfg = {}
    mats = []
    for line in refdump("config", os.path.join(REF, "config.json")):
        key, _, rest = line.partition(" ")
        if key == "material":
            n, v = rest.split()
            mats.append([n, float.fromhex(v)])
            continue
        toks = rest.split()
        vals = []
        for t in toks:
            try:
                vals.append(float.fromhex(t) if ("0x" in t) else int(t))
            except ValueError:
                vals.append(t)
        cfg[key] = vals[0] if len(vals) == 1 else vals
    cfg["materials"] = mats
    with open(os.path.join(HERE, "config_parsed.json"), "w") as fh:
        json.dump(cfg, fh, indent=1)
    # material names of the (missing) conference scene, for the synthetic stand-in
    names = []
    with open(os.path.join(REF, "conference.mtl")) as fh:
        for line in fh:
            if line.startswith("newmtl"):
                names.append(line.split()[1])
    with open(os.path.join(HERE, "conference_materials.json"), "w") as fh:
        json.dump(names, fh)
    print("fixtures written to", HERE)
    return 0


if __name__ == "__main__":
    sys.exit(main())

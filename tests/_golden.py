"""Fixture loading helpers shared by the tests (test infrastructure)."""
import json
import pathlib

import numpy as np

GOLDEN = pathlib.Path(__file__).resolve().parent / "golden"


def fixture_names():
    """SPFF-family fixtures (the 3DUNet ones are fxu3d_*: unet3d_fixture_names)."""
    return sorted(p.stem for p in GOLDEN.glob("fx*.npz") if not p.stem.startswith("fxu3d_"))


def unet3d_fixture_names():
    return sorted(p.stem for p in GOLDEN.glob("fxu3d_*.npz"))


def unet3d_state_of(d):
    """Regenerated parameters + buffers of a 3DUNet fixture (keys as in its state dict)."""
    from innovative3D.weightgen import synth_state
    shapes = d["state_shapes"]
    st = synth_state([(k, tuple(v)) for k, v in shapes.items() if k != "class_weights"],
                     d["meta"]["seed"])
    if "class_weights" in d:
        st["class_weights"] = d["class_weights"]
    return st


def load(name):
    z = np.load(GOLDEN / f"{name}.npz", allow_pickle=False)
    d = {k: z[k] for k in z.files}
    d["meta"] = json.loads(str(d["meta"]))
    d["state_shapes"] = json.loads(str(d["state_shapes"]))
    return d


def cfg_of(meta):
    from oracle.spff_oracle import SpffCfg
    kw = {k: meta[k] for k in ("efilm", "fgate", "se", "specse", "efilm_hidden", "efilm_pe_dims",
                               "learn_phase") if k in meta}
    return SpffCfg(in_ch=meta["in_ch"], num_classes=meta["K"], base=meta["base"], ksd=3, **kw)


def build_core(meta):
    """The engine-backed module tree of a non-Lightning fixture, built the way the
    fixture's generator built the reference's (make_golden.py ns_core / with_gates)."""
    import innovative3D.models as M
    fl = {k: meta.get(k, True) for k in ("efilm", "fgate", "se", "specse")}
    core = M.UNet3D_SpectralCore(in_channels=meta["in_ch"], num_classes=meta["K"], base=meta["base"],
                                 ksd=3, use_se=fl["se"], use_specse=fl["specse"])
    if fl["efilm"] or fl["fgate"]:
        core = M.upgrade_spct_with_novel_blocks(core, use_efilm=fl["efilm"], use_fouriergate=fl["fgate"])
    g = (meta.get("efilm_hidden", 32), meta.get("efilm_pe_dims", 16), meta.get("learn_phase", False))
    if g != (32, 16, False):
        for b in core._blocks():
            b.efilm = M.EnergyFiLM3D(b.efilm.channels, hidden=g[0], pe_dims=g[1])
            b.fgate = M.FourierGate3D(learn_phase=g[2])
    return core


def state_of(d):
    """Regenerate the fixture's parameters with the shared generator."""
    from innovative3D.weightgen import synth_state
    meta = d["meta"]
    shapes = d["state_shapes"]
    prefix = "model." if meta.get("lit") else ""
    st = synth_state([(k, tuple(v)) for k, v in shapes.items()], meta["seed"], meta["jitter"])
    return {k[len(prefix):] if k.startswith(prefix) else k: v for k, v in st.items()}

"""Generate the committed golden fixtures from the REFERENCE's own code.

Runs only in the build container (it reads /root/reference, which does not
exist on the GPU box).  It imports the reference modules by file path —
``useless/train.py`` (manual_pca), ``train-v4.py`` (FaceTrainer) and
``scan-template-v4.py`` (MultiModelFaceScanner) — with a minimal ``cv2``
placeholder in ``sys.modules`` because OpenCV is not installed here.  The
functions exercised never call into cv2 except ``cv2.resize`` inside
``extract_face_features``, which is handed inputs that are already 64x64
(the placeholder asserts that and returns the input unchanged).

Real-face inputs: ``faces/Light_version/*.jpg`` decoded with Pillow's
libjpeg grayscale path (``draft('L')``), which is what
``cv2.imread(..., IMREAD_GRAYSCALE)`` returns for these baseline JPEGs; the
check that this decode reproduces the reference's committed model is the
explained-variance ratio match against ``models/*_model_info.json`` below
(asserted to 1e-12).

Outputs (data only — inputs and the reference's outputs) go to
``tests/golden/*.npz``.  No reference source text is copied.

Privacy: the reference's faces are photographs of real people.  Fixtures that hold
their pixels, image-like derivatives (mean face, eigenfaces, projections) or file
names are written to ``tests/golden/local/`` only, which is git-ignored and never
committed; tests that need them skip when it is absent.  Only aggregate statistics of
the real faces (covariance eigenvalues, explained-variance ratios) are committed.

Usage:  python tests/golden/make_goldens.py
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
LOCAL = os.path.join(HERE, "local")
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))
from oracle import eigenface_oracle as orc  # noqa: E402


def _cv2_placeholder():
    m = types.ModuleType("cv2")
    m.IMREAD_GRAYSCALE = 0
    m.COLOR_BGR2GRAY = 6

    def resize(img, size, *a, **k):
        assert img.shape[:2] == (size[1], size[0]), "placeholder resize only accepts pre-sized input"
        return img

    def _absent(*a, **k):
        raise RuntimeError("cv2 is not installed in this container")

    m.resize = resize
    m.imread = m.cvtColor = m.normalize = m.imwrite = _absent
    return m


def _load(name, rel):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, rel))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def decode_dir(d):
    from PIL import Image
    files = sorted(f for f in os.listdir(d) if f.lower().endswith((".jpg", ".jpeg", ".png")))
    rows = []
    for f in files:
        im = Image.open(os.path.join(d, f))
        im.draft("L", im.size)
        rows.append(np.asarray(im.convert("L"), dtype=np.uint8).ravel())
    return np.stack(rows), files


def main():
    sys.modules.setdefault("cv2", _cv2_placeholder())
    ref_train = _load("ref_manual_train", "useless/train.py")
    ref_v4 = _load("ref_train_v4", "train-v4.py")
    ref_scan = _load("ref_scan_v4", "scan-template-v4.py")
    ref_mscan = _load("ref_manual_scan", "useless/scan.py")
    from sklearn.decomposition import PCA

    out = {}

    # ---- G1/G2: real Light faces through the reference manual_pca, k=50 -------------
    xl, files = decode_dir(os.path.join(REF, "faces/Light_version"))
    eig, mean, proj, lam = ref_train.manual_pca(xl.astype(np.float64), n_components=50)
    info_l = json.load(open(os.path.join(REF, "models/Joseph_Lai_light_model_info.json")))
    evr_l = np.array(info_l["explained_variance_ratio"])
    got = orc.manual_model_info_evr(lam)
    assert np.max(np.abs(got - evr_l)) < 1e-12, "PIL decode does not reproduce the committed light model"
    # Fix LAPACK's arbitrary eigenvector sign to the max-|.|-positive convention for storage.
    sgn = np.sign(eig[np.argmax(np.abs(eig), axis=0), np.arange(eig.shape[1])])
    os.makedirs(LOCAL, exist_ok=True)
    np.savez_compressed(  # local only: real-face pixels and image-like outputs
        os.path.join(LOCAL, "light_manual_pca.npz"),
        X=xl, k=50,
        eigenvalues=lam, mean_face=mean, projected=proj * sgn[None, :],
        eigenfaces_10=(eig[:, :10] * sgn[None, :10]).astype(np.float32),
        evr_json=evr_l,
    )
    np.savez_compressed(os.path.join(HERE, "light_stats.npz"), eigenvalues=lam, evr_json=evr_l,
                        n=xl.shape[0], d=xl.shape[1])
    o_eig, o_mean, o_proj, o_lam = orc.manual_pca(xl, 50)
    out["light oracle lam rel"] = float(np.max(np.abs(o_lam - lam) / lam))
    out["light oracle mean"] = float(np.max(np.abs(o_mean - mean)))

    # Dark: only the explained-variance ratio (the pkl is absent upstream) — store it and
    # the JSON so the CPU suite pins the oracle's EVR definition.  Faces are not stored
    # (5 MB); the oracle is checked against the reference run here.
    xd, _ = decode_dir(os.path.join(REF, "faces/Dark_version"))
    _, _, _, lam_d = ref_train.manual_pca(xd.astype(np.float64), n_components=50)
    info_d = json.load(open(os.path.join(REF, "models/Joseph_Lai_dark_model_info.json")))
    evr_d = np.array(info_d["explained_variance_ratio"])
    assert np.max(np.abs(orc.manual_model_info_evr(lam_d) - evr_d)) < 1e-12
    _, _, _, o_lam_d = orc.manual_pca(xd, 50)
    out["dark oracle lam rel"] = float(np.max(np.abs(o_lam_d - lam_d) / lam_d))
    np.savez_compressed(os.path.join(HERE, "dark_evr.npz"), eigenvalues=lam_d, evr_json=evr_d,
                        n=xd.shape[0], d=xd.shape[1])

    # ---- G3: synthetic 300x4096 uint8 -> FaceTrainer.train_pca_model (solver pinned 'full')
    xs, _ = orc.synth_faces(300, 64, r=48, seed=3)
    tr = ref_v4.FaceTrainer(n_components=16)
    tr.pca = PCA(n_components=16, svd_solver="full")
    tr.face_images = xs
    tr.face_labels = np.zeros(xs.shape[0], dtype=np.int64)
    assert tr.train_pca_model()
    p = tr.pca
    s = tr.scaler

    # ---- G4: probes through extract_face_features + recognize_face_with_model ----------
    rng = np.random.default_rng(11)
    tgt = rng.integers(0, xs.shape[0], size=24)
    probes = np.clip(np.rint(xs[tgt].astype(np.float64) + 4.0 * rng.standard_normal((24, xs.shape[1]))), 0, 255).astype(np.uint8)
    other, _ = orc.synth_faces(8, 64, r=48, seed=99)
    probes = np.concatenate([probes, other])
    labels = np.repeat(np.arange(5), 60).astype(np.int64)
    pid_map = {"alice": 0, "bob": 1, "carol": 2, "dave": 3, "erin": 4}
    md = {"scaler": s, "pca": p, "face_features": tr.face_features, "face_labels": labels,
          "person_id_map": pid_map}
    scanner = ref_scan.MultiModelFaceScanner()
    feats, pids, sims = [], [], []
    for pr in probes:
        f = scanner.extract_face_features(pr.reshape(64, 64), md)
        pid, name, sim = scanner.recognize_face_with_model(f, md, threshold=0.8)
        feats.append(f)
        pids.append(int(pid))
        sims.append(float(sim))
    np.savez_compressed(
        os.path.join(HERE, "sklearn_path.npz"),
        X=xs, k=16,
        scaler_mean=s.mean_, scaler_var=s.var_, scaler_scale=s.scale_,
        pca_mean=p.mean_, components=p.components_, explained_variance=p.explained_variance_,
        explained_variance_ratio=p.explained_variance_ratio_, singular_values=p.singular_values_,
        noise_variance=p.noise_variance_, face_features=tr.face_features, mean_face=tr.mean_face,
        probes=probes, probe_targets=np.concatenate([tgt, -np.ones(8, dtype=np.int64)]),
        probe_features=np.array(feats), labels=labels, probe_person_id=np.array(pids),
        probe_similarity=np.array(sims), threshold=0.8,
    )
    o = orc.train_pca_model(xs, 16)
    out["sk comps"] = float(np.max(np.abs(o["pca"]["components_"] - p.components_)))
    out["sk feats"] = float(np.max(np.abs(o["face_features"] - tr.face_features)))

    # ---- G5: tie-break and zero-norm cases through recognize_face_with_model ----------
    g = rng.standard_normal((40, 8))
    g[7] = g[3]            # exact duplicate: first index must win
    g[11] = 0.0            # zero-norm gallery row: similarity 0
    g[20] = 2.5 * g[3]     # same direction, larger norm: cosine tie with 3
    q = np.stack([g[3], g[3] * 0.5, np.zeros(8), 1e-3 * g[5], rng.standard_normal(8), -g[3]])
    md2 = {"face_features": g, "face_labels": np.arange(40), "person_id_map": {f"p{i}": i for i in range(40)}}
    tie_idx, tie_sim = [], []
    for qq in q:
        pid, _, sim = scanner.recognize_face_with_model(qq, md2, threshold=-2.0)
        tie_idx.append(int(pid))
        tie_sim.append(float(sim))
    np.savez_compressed(os.path.join(HERE, "ties.npz"), gallery=g, probes=q,
                        idx=np.array(tie_idx), sim=np.array(tie_sim))

    # ---- G6: manual recognize on the Light model (useless/scan.py:100-132) -------------
    mdl = {"eigenfaces": eig, "mean_face": mean, "projected_data": proj, "person_name": "Joseph_Lai"}
    noisy = np.clip(np.rint(xl[[10, 200]] + 6.0 * rng.standard_normal((2, xl.shape[1]))), 0, 255)
    flat = np.full((2, xl.shape[1]), 128.0)
    flat[1] = np.rint(mean)  # a probe equal to the mean face projects to ~0: similarity branch
    mp = np.concatenate([xl[[0, 50, 100]].astype(np.float64), noisy, flat]).astype(np.uint8)
    mres = [ref_mscan.recognize_face(v.astype(np.float64), mdl, 0.7) for v in mp]
    np.savez_compressed(os.path.join(LOCAL, "manual_scan.npz"), probes=mp,
                        sim=np.array([float(r[1]) for r in mres]),
                        recognized=np.array([bool(r[2]) for r in mres]))

    for k_, v in out.items():
        print(f"{k_}: {v:.3e}")
    make_c1_synth(ref_train, ref_mscan)


def make_c1_synth(ref_train=None, ref_mscan=None):
    """G7: config 1 without photographs — an exact-integer synthetic stand-in of
    faces/Light_version (229 x 100 x 100, so the GPU box regenerates identical pixels)
    through the reference's own ``manual_pca`` (useless/train.py:56-128),
    ``save_pca_model`` (:130-192: the pickle dict is captured in memory — nothing is
    unpickled — and the info JSON read back) and ``recognize_face`` (useless/scan.py:
    100-132)."""
    import tempfile
    sys.modules.setdefault("cv2", _cv2_placeholder())
    ref_train = ref_train or _load("ref_manual_train", "useless/train.py")
    ref_mscan = ref_mscan or _load("ref_manual_scan", "useless/scan.py")
    n, side, r, seed, k = 229, 100, 160, 7, 50
    X = orc.int_synth_faces(n, side, r=r, seed=seed)
    eig, mean, proj, lam = ref_train.manual_pca(X.astype(np.float64), n_components=k)
    captured = {}

    class _Pickle:
        @staticmethod
        def dump(obj, f, *a, **kw):
            captured["md"] = obj

    real_pickle = ref_train.pickle
    ref_train.pickle = _Pickle
    try:
        with tempfile.TemporaryDirectory() as td:
            names = [f"img_{i:03d}.png" for i in range(n)]
            ref_train.save_pca_model(eig, mean, proj, lam, names, "synth", td, "light")
            info = json.load(open(os.path.join(td, "synth_light_model_info.json")))
    finally:
        ref_train.pickle = real_pickle
    md = captured["md"]

    def describe(v):
        if isinstance(v, np.ndarray):
            return {"type": "ndarray", "dtype": str(v.dtype), "shape": list(v.shape),
                    "f_contiguous": bool(v.flags.f_contiguous), "c_contiguous": bool(v.flags.c_contiguous)}
        return {"type": type(v).__name__}

    layout = {"pkl": {key: describe(v) for key, v in md.items()}, "info_keys": sorted(info)}
    # probes: training rows, rows + integer noise, a flat face, the mean face (~0 projection)
    rng = np.random.default_rng([seed, 2])
    noisy = np.clip(X[[10, 200]].astype(np.int64) + rng.integers(-12, 13, (2, X.shape[1])), 0, 255)
    flat = np.full((1, X.shape[1]), 128)
    probes = np.concatenate([X[[0, 50, 100]], noisy, flat, np.rint(mean)[None, :]]).astype(np.uint8)
    res = [ref_mscan.recognize_face(v.astype(np.float64), md, 0.7) for v in probes]
    R = np.random.default_rng([5]).integers(0, 2, size=(X.shape[1], 8)).astype(np.float64) * 2.0 - 1.0
    sgn = np.sign(eig[np.argmax(np.abs(eig), axis=0), np.arange(k)])  # max-|.|-positive storage convention
    np.savez_compressed(
        os.path.join(HERE, "c1_synth.npz"),
        n=n, side=side, r=r, seed=seed, k=k,
        eigenvalues=lam, eigenfaces_R=(eig * sgn[None, :]).T @ R, projected=proj * sgn[None, :],
        mean_sum=mean.sum(), evr_json=np.array(info["explained_variance_ratio"]),
        layout=json.dumps(layout), probes=probes,
        sim=np.array([float(x[1]) for x in res]), recognized=np.array([bool(x[2]) for x in res]),
    )
    print("c1_synth: eigenvalues", lam[:3], "sims", [round(float(x[1]), 6) for x in res])


def make_manual_v2():
    """G8: the manual trainer's classes (scripts/manual/train-v2.py:9-72) and the manual
    scanner's helpers (useless/scan.py:58-98), imported from the reference and run on
    exact-integer synthetic faces — a Gram-shaped set (n < d) and a covariance-shaped one
    (n >= d): ManualStandardScaler.fit_transform -> ManualPCA(k).fit_transform, plus
    ManualPCA.transform / project_face_to_eigenspace of probes and cosine_similarity of
    vector pairs (including a zero vector)."""
    sys.modules.setdefault("cv2", _cv2_placeholder())
    ref_m = _load("ref_manual_train_v2", "scripts/manual/train-v2.py")
    ref_mscan = _load("ref_manual_scan", "useless/scan.py")
    res = {}
    for tag, (n, side, r, seed, k) in {"gram": (150, 20, 40, 21, 20), "cov": (400, 16, 40, 22, 24)}.items():
        X = orc.int_synth_faces(n, side, r=r, seed=seed)
        sc = ref_m.ManualStandardScaler()
        Z = sc.fit_transform(X.astype(np.float64))
        pca = ref_m.ManualPCA(n_components=k)
        F = pca.fit_transform(Z)
        sgn = np.sign(pca.components_[np.arange(k), np.argmax(np.abs(pca.components_), axis=1)])
        probes = np.clip(X[:6].astype(np.int64) + np.random.default_rng(seed).integers(-9, 10, (6, X.shape[1])),
                         0, 255).astype(np.uint8)
        Fp = pca.transform(sc.transform(probes.astype(np.float64)))
        # the manual scanner's projection with (d, k) eigenfaces, raw pixels
        E = (pca.components_ * sgn[:, None]).T
        P = np.stack([ref_mscan.project_face_to_eigenspace(v.astype(np.float64), E, sc.mean_) for v in probes])
        res.update({f"{tag}_n": n, f"{tag}_side": side, f"{tag}_r": r, f"{tag}_seed": seed, f"{tag}_k": k,
                    f"{tag}_scaler_mean": sc.mean_, f"{tag}_scaler_scale": sc.scale_,
                    f"{tag}_components": pca.components_ * sgn[:, None],
                    f"{tag}_evr": pca.explained_variance_ratio_, f"{tag}_features": F * sgn[None, :],
                    f"{tag}_probes": probes, f"{tag}_probe_features": Fp * sgn[None, :],
                    f"{tag}_projected": P})
        o_c, o_m, o_evr, _, o_f = orc.manual_pca_cov(orc.manual_standard_scaler(X)[0], k)
        print(tag, "oracle vs reference: comps", float(np.max(np.abs(o_c - pca.components_ * sgn[:, None]))),
              "evr", float(np.max(np.abs(o_evr - pca.explained_variance_ratio_))))
    rng = np.random.default_rng(31)
    a = rng.standard_normal((6, 50))
    b = rng.standard_normal((6, 50))
    b[1] = 3.0 * a[1]       # parallel: similarity 1
    b[2] = -a[2]            # anti-parallel: -1
    a[3] = 0.0              # zero vector: 0.0 (:73-74)
    b[4] = a[4] + 1e-9      # near-identical
    cs = np.array([ref_mscan.cosine_similarity(x, y) for x, y in zip(a, b)], dtype=np.float64)
    res.update(cos_a=a, cos_b=b, cos_sim=cs)
    np.savez_compressed(os.path.join(HERE, "manual_v2.npz"), **res)
    print("manual_v2: cos", cs)


def _fit_summary(eig, proj, lam, d, n_rows=64):
    """Compact, sign-normalised summary of a manual_pca result (eig: d x k columns).
    Signs: largest |entry| positive (first on ties), the svd_flip rule the GPU fit
    applies (LAPACK's eigh signs are arbitrary); top_idx / top_val keep each component's
    two largest |entries| so a test can tell a near-tied (legitimately flippable) sign."""
    k = eig.shape[1]
    sgn = np.sign(eig[np.argmax(np.abs(eig), axis=0), np.arange(k)])
    comps = (eig * sgn[None, :]).T
    R = np.random.default_rng([5]).integers(0, 2, size=(d, 8)).astype(np.float64) * 2.0 - 1.0
    px = np.sort(np.random.default_rng([6]).choice(d, size=256, replace=False))
    top_idx = np.argsort(-np.abs(comps), axis=1, kind="stable")[:, :2]
    return dict(eigenvalues=lam, comps_R=comps @ R, comps_px=comps[:, px], px=px,
                top_idx=top_idx, top_val=np.take_along_axis(comps, top_idx, axis=1),
                projected=(proj * sgn[None, :])[:n_rows], proj_colnorm=np.linalg.norm(proj, axis=0))


def make_fit_shapes():
    """G9 (VERDICT r3 "next" 3): the reference's own ``manual_pca`` (useless/train.py:
    56-128), imported and run here, on two exact-integer synthetic sets the GPU box
    regenerates bit for bit:

    * ``fit_c2.npz`` — BASELINE.json configs[1]'s fit shape: n = 10000, d = 128 x 128 =
      16384, k = 64: the Gram path at order 10000 (A.A^T, eigh, A^T.V back-projection);
    * ``fit_hard.npz`` — a Light-like set: n = 229, d = 100 x 100 (faces/Light_version's
      shape), factor weights from the real Light eigenvalue profile
      (``light_like_spectrum`` of light_stats.npz), so the sample spectrum has the real
      set's clustered eigen-gaps (min relative gap ~1 %); all 50 components are compared
      at the north star's 1e-4.
    """
    import time
    sys.modules.setdefault("cv2", _cv2_placeholder())
    ref_train = _load("ref_manual_train", "useless/train.py")
    # hard spectrum
    lam_light = np.load(os.path.join(HERE, "light_stats.npz"))["eigenvalues"]
    n, side, r, seed, k = 229, 100, 228, 8, 50
    spec = orc.light_like_spectrum(lam_light, r)
    X = orc.int_synth_faces(n, side, r=r, seed=seed, spectrum=spec)
    eig, mean, proj, lam = ref_train.manual_pca(X.astype(np.float64), n_components=k)
    np.savez_compressed(os.path.join(HERE, "fit_hard.npz"), n=n, side=side, r=r, seed=seed, k=k, spectrum=spec,
                        mean_sum=mean.sum(), **_fit_summary(eig, proj, lam, side * side))
    g = -np.diff(lam) / lam[:-1]
    print("fit_hard: lam", lam[:3], "min rel gap", float(g.min()))
    # C2 fit shape
    n, side, r, seed, k = 10000, 128, 160, 3, 64
    X = orc.int_synth_faces(n, side, r=r, seed=seed)
    t = time.time()
    eig, mean, proj, lam = ref_train.manual_pca(X.astype(np.float64), n_components=k)
    print(f"fit_c2: reference manual_pca {time.time() - t:.0f} s; lam", lam[:3], lam[-1])
    np.savez_compressed(os.path.join(HERE, "fit_c2.npz"), n=n, side=side, r=r, seed=seed, k=k,
                        mean_sum=mean.sum(), **_fit_summary(eig, proj, lam, side * side))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "c1":
        make_c1_synth()
    elif len(sys.argv) > 1 and sys.argv[1] == "manual_v2":
        make_manual_v2()
    elif len(sys.argv) > 1 and sys.argv[1] == "fit_shapes":
        make_fit_shapes()
    else:
        main()

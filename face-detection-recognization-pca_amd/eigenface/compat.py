"""On-disk formats and the trainer/scanner surface of the reference (SURVEY.md
Appendix A, §8a rows a1/a10/a11), backed by the GPU engine.

* ``FaceTrainer``            — train-v4.py:11-266 (load, label, train, save/load model,
                               eigenface JPGs + ``{person}_model_info.json``)
* ``save_pca_model``         — useless/train.py:130-192 (``models/*_pca_model.pkl`` +
                               ``*_model_info.json``)
* ``visualize_eigenfaces``   — useless/train.py:194-223
* ``sklearn_objects``        — real ``StandardScaler`` / ``PCA`` instances populated from the
                               GPU fit, so pickles load and ``.transform`` anywhere sklearn
                               is installed (scan-template-v4.py:36-37, :265-266)
* ``extract_face_features``, ``recognize_face_all_models`` — scan-template-v4.py:253-319

Image ingest (a1, §8f rank 2): JPEG files are decoded on the GPU in one batch with
libjpeg-turbo's arithmetic (``ef_jpeg_ingest`` / ``ef_jpeg_decode``, bit-exact against
Pillow's libjpeg-turbo — the library cv2.imread wraps), then ``cvtColor(BGR2GRAY)`` +
``resize(64, 64)`` run in the same call with OpenCV's CV_8U fixed-point rules (*parity
unpinned* against OpenCV itself, which is absent where this was built).  Files
the GPU decoder does not take (PNG, progressive/CMYK JPEG) are decoded on the host by
OpenCV or Pillow and join the GPU grey+resize launch.
"""
from __future__ import annotations

import json
import os
import pickle
from datetime import datetime

import numpy as np

from ._native import EigenfaceError
from .pca import EigenfacePCA, _model_engine, get_engine


# ----------------------------------------------------------------------- images
def decode_image(path):
    """cv2.imread(path) (IMREAD_COLOR, BGR uint8) or None if unreadable.  Decoding is
    libjpeg either way: OpenCV when importable, else Pillow (RGB reversed to BGR)."""
    try:
        import cv2
    except ImportError:
        cv2 = None
    if cv2 is not None:
        return cv2.imread(path)
    try:
        from PIL import Image
        im = Image.open(path)
        if im.mode == "L":
            return np.asarray(im, dtype=np.uint8)
        return np.ascontiguousarray(np.asarray(im.convert("RGB"), dtype=np.uint8)[..., ::-1])
    except (OSError, ValueError):
        return None


def _read_bytes(path):
    try:
        with open(path, "rb") as f:
            return f.read()
    except OSError:
        return None


def _is_jpeg(blob):
    return blob is not None and len(blob) > 3 and blob[0] == 0xFF and blob[1] == 0xD8


def read_faces(paths, size=(64, 64), device=0):
    """train-v4.py:59-68 for a list of files: JPEG files are decoded, converted to grey
    and resized on the GPU in one batch (ef_jpeg_ingest; libjpeg-turbo's IMREAD_COLOR
    pixels, then cvtColor(BGR2GRAY) + resize(size)); files the GPU decoder does not take
    (PNG, progressive or CMYK JPEG) are decoded on the host by the reference's own decoder
    and join one GPU grey+resize launch (ef_preprocess).  Returns (rows uint8 (m, h*w),
    kept indices) — unreadable files are skipped like the reference's ``img is None``
    branch."""
    eng = get_engine(device)
    blobs = [_read_bytes(p) for p in paths]
    jpg = [i for i, b in enumerate(blobs) if _is_jpeg(b)]
    rows = {}
    if jpg:
        r, st = eng.ingest_jpegs([blobs[i] for i in jpg], size, "bgr")
        for k, i in enumerate(jpg):
            if st[k] == 0:
                rows[i] = r[k]
    rest, imgs = [], []
    for i, p in enumerate(paths):
        if i in rows or blobs[i] is None:
            continue
        im = decode_image(p)
        if im is not None:
            rest.append(i)
            imgs.append(im)
    if imgs:
        for i, r in zip(rest, eng.preprocess(imgs, size)):
            rows[i] = r
    keep = sorted(rows)
    if not keep:
        return np.zeros((0, size[0] * size[1]), np.uint8), keep
    return np.stack([rows[i] for i in keep]), keep


def read_gray_images(paths, device=0):
    """cv2.imread(path, IMREAD_GRAYSCALE) for a list of files (useless/train.py:33,
    scan-template-v4.py:52): JPEGs decoded on the GPU in one batch (libjpeg's grey output),
    other files by decode_gray on the host.  Returns a list of uint8 arrays (None for an
    unreadable file)."""
    blobs = [_read_bytes(p) for p in paths]
    jpg = [i for i, b in enumerate(blobs) if _is_jpeg(b)]
    out = [None] * len(paths)
    if jpg:
        for i, im in zip(jpg, get_engine(device).decode_jpegs([blobs[i] for i in jpg], "gray")):
            out[i] = im
    for i, p in enumerate(paths):
        if out[i] is None and blobs[i] is not None:
            out[i] = decode_gray(p)
    return out


def read_face(path, size=(64, 64), device=0):
    """Grey, resized, uint8 face (train-v4.py:59-66); None if unreadable."""
    rows, keep = read_faces([path], size, device)
    return rows[0].reshape(size[1], size[0]) if keep else None


def _save_bgr_jpg(path, bgr):
    """cv2.imwrite of a BGR (or grey) uint8 crop (detection-v4.py:64)."""
    a = np.ascontiguousarray(bgr, dtype=np.uint8)
    try:
        import cv2
        cv2.imwrite(path, a)
    except ImportError:
        from PIL import Image
        Image.fromarray(a[..., ::-1] if a.ndim == 3 else a).save(path, quality=95)


def _save_jpg(path, arr2d, truncate=False):
    """cv2.normalize(NORM_MINMAX, 0..255, CV_8U) + imwrite (train-v4.py:164-177); with
    ``truncate`` the float normalize + astype(uint8) of useless/train.py:205-216."""
    a = np.asarray(arr2d, dtype=np.float64)
    lo, hi = a.min(), a.max()
    if hi == lo:
        u8 = np.zeros(a.shape, np.uint8)
    else:
        v = (a - lo) * (255.0 / (hi - lo))
        u8 = (np.floor(v) if truncate else np.rint(v)).astype(np.uint8)
    try:
        import cv2
        cv2.imwrite(path, u8)
    except ImportError:
        from PIL import Image
        Image.fromarray(u8, mode="L").save(path, quality=95)


# ------------------------------------------------------------ sklearn objects
def sklearn_objects(model: EigenfacePCA):
    """Fitted ``StandardScaler`` and ``PCA`` carrying the GPU fit's attributes."""
    from sklearn.decomposition import PCA
    from sklearn.preprocessing import StandardScaler

    d = model.n_features_in_
    scaler = StandardScaler()
    if model.standardize:
        scaler.mean_, scaler.var_, scaler.scale_ = model.scaler_mean_.copy(), model.scaler_var_.copy(), \
            model.scaler_scale_.copy()
    else:  # identity scaling: the PCA is on raw pixels (manual_pca semantics)
        scaler.mean_, scaler.var_, scaler.scale_ = np.zeros(d), np.ones(d), np.ones(d)
    scaler.n_samples_seen_ = model.n_samples_
    scaler.n_features_in_ = d
    pca = PCA(n_components=model.n_components, svd_solver="full")
    pca.mean_ = model.mean_.copy()
    pca.components_ = model.components_.copy()
    pca.explained_variance_ = model.explained_variance_.copy()
    pca.explained_variance_ratio_ = model.explained_variance_ratio_.copy()
    pca.singular_values_ = model.singular_values_.copy()
    pca.noise_variance_ = model.noise_variance_
    pca.n_components_ = model.n_components_
    pca.n_samples_ = model.n_samples_
    pca.n_features_in_ = d
    pca._fit_svd_solver = "full"
    return scaler, pca


# ------------------------------------------------------------------ trainer
class FaceTrainer:
    """train-v4.py's FaceTrainer (:11-266) with the fit on the GPU."""

    def __init__(self, n_components=50, device=0):
        self.n_components = n_components
        self.device = device
        self.pca = None
        self.scaler = None
        self.face_features = []
        self.face_labels = []
        self.face_info = []
        self.face_images = np.zeros((0, 0), np.uint8)
        self.person_id_map = {}
        self.is_trained = False
        self.mean_face = None
        self.eigenfaces = None
        self.face_shape = (64, 64)
        self.model = None

    def load_face_images(self, json_path, face_dir):
        """JSON order (train-v4.py:44-76).  ``image_path`` as the reference, falling back to
        ``image_filename`` inside face_dir (train-v5.py:305-306) for Windows-style paths."""
        with open(json_path, "r", encoding="utf-8") as f:
            data = json.load(f)
        paths, infos = [], []
        for info in data["faces"]:
            path = info.get("image_path", "")
            if not os.path.exists(path):
                alt = os.path.join(face_dir, info.get("image_filename", os.path.basename(path.replace("\\", "/"))))
                if not os.path.exists(alt):
                    print(f"Warning: Image {path} not found, skipping...")
                    continue
                path = alt
            paths.append(path)
            infos.append(info)
        rows, keep = read_faces(paths, self.face_shape, self.device)
        for i in sorted(set(range(len(paths))) - set(keep)):
            print(f"Warning: Could not read image {paths[i]}, skipping...")
        self.face_images = rows
        self.face_info = [infos[i] for i in keep]
        return len(keep)

    def assign_labels_interactive(self, person_name):
        """All faces labelled as one person, id 0 (train-v4.py:78-108)."""
        for info in self.face_info:
            info["person_name"] = person_name
            info["person_id"] = 0
        self.face_labels = np.zeros(len(self.face_info), dtype=np.int64)
        self.person_id_map = {person_name: 0}
        return list(self.face_labels)

    def train_pca_model(self):
        """StandardScaler -> PCA on the GPU (train-v4.py:110-146); False on empty input."""
        if len(self.face_images) == 0:
            print("Error: No face images loaded!")
            return False
        if len(self.face_labels) == 0:
            print("Error: No face labels assigned!")
            return False
        try:
            m = EigenfacePCA(self.n_components, standardize=True, device=self.device).fit(self.face_images)
        except EigenfaceError as e:  # e.g. EF_E_NUMERIC: eigensolver did not converge
            print(f"Error: PCA training failed: {e}")
            return False
        self.model = m
        self.mean_face = m.mean_face_
        self.scaler, self.pca = sklearn_objects(m)
        self.eigenfaces = self.pca.components_
        self.face_features = m.face_features_
        print(f"PCA explained variance ratio: {self.pca.explained_variance_ratio_.sum():.3f}")
        self.is_trained = True
        return True

    def save_eigenfaces(self, output_dir, person_name):
        """Mean face + top-10 eigenfaces as min-max JPGs and ``{person}_model_info.json``
        (train-v4.py:148-197)."""
        if not self.is_trained:
            print("Error: Model not trained yet!")
            return False
        os.makedirs(output_dir, exist_ok=True)
        _save_jpg(os.path.join(output_dir, f"{person_name}_mean_face.jpg"), self.mean_face.reshape(self.face_shape))
        n_save = min(10, len(self.eigenfaces))
        for i in range(n_save):
            _save_jpg(os.path.join(output_dir, f"{person_name}_eigenface_{i + 1:02d}.jpg"),
                      self.eigenfaces[i].reshape(self.face_shape))
        info = {
            "person_name": person_name,
            "training_date": datetime.now().isoformat(),
            "total_faces": len(self.face_images),
            "n_components": self.n_components,
            "explained_variance_ratio": float(self.pca.explained_variance_ratio_.sum()),
            "face_shape": self.face_shape,
            "eigenfaces_saved": n_save,
        }
        with open(os.path.join(output_dir, f"{person_name}_model_info.json"), "w", encoding="utf-8") as f:
            json.dump(info, f, indent=2, ensure_ascii=False)
        return True

    def model_dict(self):
        """The ``face_model.pkl`` dict (train-v4.py:210-222)."""
        return {
            "pca": self.pca,
            "scaler": self.scaler,
            "face_features": self.face_features,
            "face_labels": self.face_labels,
            "face_info": self.face_info,
            "person_id_map": self.person_id_map,
            "n_components": self.n_components,
            "mean_face": self.mean_face,
            "eigenfaces": self.eigenfaces,
            "face_shape": self.face_shape,
            "training_date": datetime.now().isoformat(),
        }

    def save_model(self, model_path):
        if not self.is_trained:
            print("Error: Model not trained yet!")
            return False
        with open(model_path, "wb") as f:
            pickle.dump(self.model_dict(), f)
        return True

    def load_model(self, model_path):
        """Load a model this package (or the reference) wrote — trusted files only: a
        pickle executes code on load."""
        if not os.path.exists(model_path):
            print(f"Error: Model file {model_path} not found!")
            return False
        with open(model_path, "rb") as f:
            md = pickle.load(f)
        self.pca = md["pca"]
        self.scaler = md["scaler"]
        self.face_features = md["face_features"]
        self.face_labels = md["face_labels"]
        self.face_info = md["face_info"]
        self.person_id_map = md["person_id_map"]
        self.n_components = md["n_components"]
        self.mean_face = md.get("mean_face")
        self.eigenfaces = md.get("eigenfaces")
        self.face_shape = md.get("face_shape", (64, 64))
        self.is_trained = True
        return True


# ----------------------------------------------------------- manual formats
def save_pca_model(eigenfaces, mean_face, projected_data, eigenvalues, filenames, person_name, model_dir,
                   version=None):
    """``models/{person}[_{version}]_pca_model.pkl`` + ``_model_info.json``
    (useless/train.py:130-192).  The JSON ratio divides by the sum of the *kept*
    eigenvalues and keeps the first 10 (:182)."""
    os.makedirs(model_dir, exist_ok=True)
    stamp = datetime.now().isoformat()
    md = {
        "eigenfaces": eigenfaces,
        "mean_face": mean_face,
        "projected_data": projected_data,
        "eigenvalues": eigenvalues,
        "training_filenames": list(filenames),
        "person_name": person_name,
        "version": version,
        "training_timestamp": stamp,
        "n_components": int(eigenfaces.shape[1]),
        "face_dimensions": int(eigenfaces.shape[0]),
    }
    stem = f"{person_name}_{version}" if version else person_name
    model_file = f"{stem}_pca_model.pkl"
    path = os.path.join(model_dir, model_file)
    with open(path, "wb") as f:
        pickle.dump(md, f)
    lam = np.asarray(eigenvalues, dtype=np.float64)
    meta = {
        "person_name": person_name,
        "version": version,
        "training_timestamp": stamp,
        "n_components": md["n_components"],
        "face_dimensions": md["face_dimensions"],
        "n_training_images": len(filenames),
        "explained_variance_ratio": (lam / lam.sum()).tolist()[:10],
        "model_file": model_file,
    }
    with open(os.path.join(model_dir, f"{stem}_model_info.json"), "w", encoding="utf-8") as f:
        json.dump(meta, f, indent=2, ensure_ascii=False)
    return path


def visualize_eigenfaces(eigenfaces, mean_face, output_dir, person_name, n_display=10):
    """Mean face + top eigenfaces as min-max JPGs (useless/train.py:194-223)."""
    side = int(np.sqrt(len(mean_face)))
    _save_jpg(os.path.join(output_dir, f"{person_name}_mean_face.jpg"), np.asarray(mean_face).reshape(side, side),
              truncate=True)
    for i in range(min(n_display, eigenfaces.shape[1])):
        _save_jpg(os.path.join(output_dir, f"{person_name}_eigenface_{i + 1:02d}.jpg"),
                  eigenfaces[:, i].reshape(side, side), truncate=True)


# ------------------------------------------------------------------ scanner
def _model_projection(md):
    """Fold a face_model.pkl's scaler + pca into (mean, W) for the GPU projection.  The
    estimator is read from ``md['pca']`` only, as scan-template-v4.py:266 does: a model
    dict without that key (the reference's own faces/lock_version/Joseph_Lai/face_model.pkl
    is keyed ``pca_model``) raises ``KeyError('pca')``, which the per-model ``try`` of
    recognize_faces_all_models reports and skips, exactly as the reference (:312-314)."""
    pca = md["pca"]
    sc = md["scaler"]
    comp = np.asarray(pca.components_, dtype=np.float64)
    scale = np.asarray(sc.scale_, dtype=np.float64)
    w = (comp / scale[None, :]).T
    mu = np.asarray(sc.mean_, dtype=np.float64) + scale * np.asarray(pca.mean_, dtype=np.float64)
    return mu.astype(np.float32), np.ascontiguousarray(w, dtype=np.float32)


_fold_cache: dict = {}


def _folded(md):
    """(mean, W) of a model dict, folded once per model (the cache keeps the dict and the
    estimator arrays it was folded from, so a replaced or refitted estimator re-folds)."""
    pca = md["pca"]  # no fallback key: see _model_projection
    sc = md["scaler"]
    src = (pca.components_, pca.mean_, sc.mean_, sc.scale_)
    hit = _fold_cache.get(id(md))
    if hit is not None and hit[0] is md and all(x is y for x, y in zip(hit[1], src)):
        return hit[2], hit[3]
    mu, w = _model_projection(md)
    if len(_fold_cache) > 64:
        _fold_cache.clear()
    _fold_cache[id(md)] = (md, src, mu, w)
    return mu, w


def preprocess_faces(face_imgs, device=0):
    """Grey 64x64 rows of a batch of face crops (scan-template-v4.py:257-263): one GPU
    launch (ef_preprocess) for the whole batch."""
    return get_engine(device).preprocess([np.asarray(f, dtype=np.uint8) for f in face_imgs], (64, 64))


def extract_faces_features(face_rows, model_data, device=0):
    """scan-template-v4.py:253-268 for a batch: ``face_rows`` (b, 4096) uint8 from
    :func:`preprocess_faces` -> (b, k) features (one projection launch)."""
    mu, w = _folded(model_data)
    eng = _model_engine(mu, w, device)
    return eng.project(np.asarray(face_rows)).astype(np.float64)


def extract_face_features(face_img, model_data, device=0):
    """scan-template-v4.py:253-268 on the GPU: grey face crop -> model features."""
    return extract_faces_features(preprocess_faces([face_img], device), model_data, device)[0]


def recognize_faces_all_models(face_imgs, models, threshold=0.8, device=0):
    """recognize_face_all_models (scan-template-v4.py:289-319) for every detection of a
    frame at once: the crops are preprocessed in one launch, then per model one projection
    and one cosine search over all of them.  Per face: strict '>' over models in
    iteration order, the recognised name or the model's person name; (-1, "unknown", 0.0)
    when no model scores above 0."""
    from .pca import _gallery_engine

    n = len(face_imgs)
    best = [None] * n
    best_conf = np.zeros(n)
    if n == 0:
        return []
    # one launch for the batch; if a crop is unusable (the reference's per-face resize
    # raises inside the per-model try, :312-314), find it and give it the sentinel
    try:
        rows = preprocess_faces(face_imgs, device)
        ok = np.arange(n)
    except Exception:  # noqa: BLE001
        good, parts = [], []
        for i, img in enumerate(face_imgs):
            try:
                parts.append(preprocess_faces([img], device))
                good.append(i)
            except Exception as e:  # noqa: BLE001
                print(f"Error recognizing face {i}: {e}")
        if not good:
            return [(-1, "unknown", 0.0)] * n
        rows, ok = np.concatenate(parts), np.asarray(good)
    for person_name, info in models.items():
        md = info["model_data"] if "model_data" in info else info
        if md is None:
            continue
        try:  # everything per model inside the try, as the reference (:302-314)
            f = extract_faces_features(rows, md, device)
            eng = _gallery_engine(md["face_features"], device)
            idx, sim = eng.search(f.astype(np.float32), "cosine")
            labels, pmap = md["face_labels"], md["person_id_map"]
            upd = []
            for j, i in enumerate(ok):
                conf = float(sim[j])
                if not conf > best_conf[i]:
                    continue
                pid, name = -1, "unknown"
                if idx[j] >= 0 and conf >= threshold:  # recognize_face_with_model (:278-284)
                    pid = labels[idx[j]]
                    for nm, v in pmap.items():
                        if v == pid:
                            name = nm
                            break
                upd.append((i, conf, (pid, name if name != "unknown" else person_name, conf)))
        except Exception as e:  # reference: print and continue (:312-314)
            print(f"Error recognizing with model {person_name}: {e}")
            continue
        for i, conf, rec in upd:  # a model that fails half-way changes nothing
            best_conf[i] = conf
            best[i] = rec
    return [b if b else (-1, "unknown", 0.0) for b in best]


def recognize_face_all_models(face_img, models, threshold=0.8, device=0):
    """Best match over per-person models for one face (scan-template-v4.py:289-319)."""
    return recognize_faces_all_models([face_img], models, threshold, device)[0]


def load_all_models(root="."):
    """``MultiModelFaceScanner.load_all_models`` (scan-template-v4.py:17-74): every
    ``faces/lock_version/*/face_model.pkl`` under ``root`` (glob order, sorted here for
    determinism), keyed by the person directory name, each entry
    ``{model_data, detection_data, template_images, model_path}`` with up to 5 templates
    ``{image (grey, IMREAD_GRAYSCALE), width, height}`` from the first faces of
    ``{person}_faces_detection.json`` whose ``image_path`` exists (:48-58).  Models that
    fail to load are reported and skipped (:70-71).  Pickles execute code when loaded:
    only load model files you trust."""
    import glob

    models = {}
    pattern = os.path.join(root, "faces", "lock_version", "*", "face_model.pkl")
    paths = sorted(glob.glob(pattern))
    if not paths:
        print(f"No models found matching pattern: {pattern}")
        return models
    print(f"Found {len(paths)} model(s):")
    for model_path in paths:
        person_name = os.path.basename(os.path.dirname(model_path))
        try:
            with open(model_path, "rb") as f:
                md = pickle.load(f)
            json_path = os.path.join(os.path.dirname(model_path), f"{person_name}_faces_detection.json")
            det = None
            if os.path.exists(json_path):
                with open(json_path, "r", encoding="utf-8") as f:
                    det = json.load(f)
            templates = []
            if det and det.get("faces"):
                first = [f for f in det["faces"][:5] if os.path.exists(f["image_path"])]
                for face, img in zip(first, read_gray_images([f["image_path"] for f in first])):
                    if img is not None:
                        templates.append({"image": img, "width": face["width"], "height": face["height"]})
            models[person_name] = {"model_data": md, "detection_data": det, "template_images": templates,
                                   "model_path": model_path}
            print(f"  - {person_name}: {len(md['face_features']) if md else 0} faces")
        except Exception as e:  # noqa: BLE001 - the reference prints and continues
            print(f"  - Failed to load {person_name}: {e}")
    print(f"Successfully loaded {len(models)} model(s)")
    return models


def decode_gray(path):
    """cv2.imread(path, IMREAD_GRAYSCALE): libjpeg's grey output (OpenCV when importable,
    else Pillow's draft('L') — the decode pinned by the reference models' EVR); None if
    unreadable."""
    try:
        import cv2
    except ImportError:
        cv2 = None
    if cv2 is not None:
        return cv2.imread(path, cv2.IMREAD_GRAYSCALE)
    try:
        from PIL import Image
        im = Image.open(path)
        im.draft("L", im.size)
        return np.asarray(im.convert("L"), dtype=np.uint8)
    except (OSError, ValueError):
        return None

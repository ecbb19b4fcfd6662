"""Drop-in command lines for the training scripts, with the fit on the GPU.

    python -m eigenface.cli train --person NAME
        train-v4.py main (:268-312): faces/lock_version/NAME/NAME_faces_detection.json ->
        face_model.pkl + eigenface JPGs + NAME_model_info.json (what run_pipeline.py:234 runs)

    python -m eigenface.cli train-manual --faces-dir DIR --person NAME [--version V]
        useless/train.py train_single_model (:225-276): sorted images of DIR ->
        models/NAME[_V]_pca_model.pkl + _model_info.json + JPGs

    python -m eigenface.cli train-v5 [--base-dir faces/lock_version]
        train-v5.py main (:570-610): one full-rank model per person directory

The reference-named entry files ``face-detection-recognization-pca_amd/dropin/train-v4.py``
and ``train-v5.py`` wrap these for unchanged callers (run_pipeline.py:234).
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np


def train_v4(person, root="."):
    """train-v4.py main (:268-312); returns True when a model was written."""
    from .compat import FaceTrainer

    json_path = os.path.join(root, f"faces/lock_version/{person}/{person}_faces_detection.json")
    face_dir = os.path.join(root, f"faces/lock_version/{person}")
    model_path = os.path.join(face_dir, "face_model.pkl")
    if not os.path.exists(json_path):
        print(f"Error: JSON file {json_path} not found!")
        print("Please run detection-v2.py first to generate face data.")
        return False
    tr = FaceTrainer(n_components=50)
    if tr.load_face_images(json_path, face_dir) == 0:
        print("No valid face images found!")
        return False
    if len(tr.assign_labels_interactive(person)) == 0:
        print("No faces labeled, training cancelled.")
        return False
    if not tr.train_pca_model():
        print("Training failed!")
        return False
    tr.save_eigenfaces(face_dir, person)
    tr.save_model(model_path)
    print(f"\nTraining completed successfully!\nModel saved to: {model_path}")
    print(f"Eigenfaces and mean face saved to: {face_dir}")
    return True


def train_manual(faces_dir, person, model_dir="models", version=None, n_components=50):
    from .compat import read_face, save_pca_model, visualize_eigenfaces
    from .pca import manual_pca

    from .compat import read_gray_images

    files = sorted(f for f in os.listdir(faces_dir) if f.lower().endswith((".jpg", ".jpeg", ".png")))
    rows, names = [], []
    # cv2.imread(IMREAD_GRAYSCALE) per file (useless/train.py:33): JPEGs decoded on the GPU
    # in one batch (libjpeg's grey output, pinned by the reference models' EVR)
    for f, im in zip(files, read_gray_images([os.path.join(faces_dir, f) for f in files])):
        if im is None:
            print(f"Warning: Could not load image {f}")
            continue
        rows.append(np.ascontiguousarray(im, dtype=np.uint8).ravel())
        names.append(f)
    if not rows:
        print("Error: No valid face images could be loaded")
        return 1
    X = np.stack(rows)
    eig, mean, proj, lam = manual_pca(X, n_components)
    save_pca_model(eig, mean, proj, lam, names, person, model_dir, version)
    visualize_eigenfaces(eig, mean, model_dir, f"{person}_{version}" if version else person)
    print(f"Training images: {len(names)}  components: {eig.shape[1]}  dims: {eig.shape[0]}")
    return 0


def main(argv=None):
    ap = argparse.ArgumentParser(prog="eigenface.cli")
    sub = ap.add_subparsers(dest="cmd", required=True)
    t = sub.add_parser("train", help="train-v4.py drop-in")
    t.add_argument("--person", required=True)
    t.add_argument("--root", default=".")
    m = sub.add_parser("train-manual", help="useless/train.py drop-in (one version)")
    m.add_argument("--faces-dir", required=True)
    m.add_argument("--person", required=True)
    m.add_argument("--model-dir", default="models")
    m.add_argument("--version", default=None)
    m.add_argument("--k", type=int, default=50)
    v5 = sub.add_parser("train-v5", help="train-v5.py drop-in (every person directory)")
    v5.add_argument("--base-dir", default="faces/lock_version")
    a = ap.parse_args(argv)
    if a.cmd == "train":
        return 0 if train_v4(a.person, a.root) else 1
    if a.cmd == "train-v5":
        from .multi_person import main as v5_main
        ok, failed = v5_main(a.base_dir)
        return 0 if ok and not failed else 1
    return train_manual(a.faces_dir, a.person, a.model_dir, a.version, a.k)


def main_train_v4():
    """train-v4.py's command line; like the reference's main it exits 0 after printing
    an error (run_pipeline.py:41 only sees crashes)."""
    ap = argparse.ArgumentParser(description="Train face recognition model using PCA")
    ap.add_argument("--person", required=True, help="Person name for training model")
    train_v4(ap.parse_args().person)


if __name__ == "__main__":
    sys.exit(main())

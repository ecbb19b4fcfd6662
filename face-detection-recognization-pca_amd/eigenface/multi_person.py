"""train-v5.py's per-person trainer with the fit on the GPU.

* ``MultiFaceTrainer``        — train-v5.py:13-505: detection-JSON synthesis from a directory
                                of crops, face counting, JSON / all-person loading, the
                                StandardScaler + PCA fit, ``multi_person_*`` artefacts
* ``train_person_model``      — train-v5.py:507-568: one model per person directory with
                                ``n_components = face_count`` (full rank, k = n)
* ``main``                    — train-v5.py:570-610: every directory of faces/lock_version

Differences from the reference, all deliberate and documented:
* the fit is ``EigenfacePCA(k, standardize=True)`` (deterministic; with k = n sklearn's
  ``auto`` solver is already the deterministic ``full`` one, _pca.py:524-536);
* the numerically null last component of a k = n fit (the centred data has rank n - 1)
  is a fixed unit vector orthogonal to the data span (include/eigenface.h ef_fit), where
  sklearn returns LAPACK's arbitrary choice — parity for that one component is unpinned;
* crops are decoded on the host (libjpeg) and grey + resize run as one GPU launch per
  person (ef_preprocess, OpenCV CV_8U rules; parity against OpenCV unpinned).
"""
from __future__ import annotations

import glob
import json
import os
import pickle
import re
from datetime import datetime

import numpy as np

from ._native import EigenfaceError
from .compat import _save_jpg, decode_image, read_faces, sklearn_objects
from .pca import EigenfacePCA

_SKIP = ("eigenface", "mean_face", "model_info")


class MultiFaceTrainer:
    """train-v5.py MultiFaceTrainer (:13-505) with the fit on the GPU."""

    def __init__(self, n_components=50, device=0):
        self.n_components = n_components
        self.device = device
        self.pca = None
        self.scaler = None
        self.face_features = []
        self.face_labels = []
        self.face_info = []
        self.face_images = np.zeros((0, 0), np.uint8)
        self.is_trained = False
        self.mean_face = None
        self.eigenfaces = None
        self.face_shape = (64, 64)
        self.person_id_map = {}
        self.model = None

    # ------------------------------------------------------------ detection JSON
    def generate_detection_json_for_person(self, person_name, face_dir):
        """{person}_faces_detection.json synthesised from the crops in face_dir
        (train-v5.py:33-142): sorted unique files of the three glob patterns, frame
        number from ``face_N_frame_F`` / ``_face_N`` names, timestamps at 30 fps, the
        crop's size (64 x 64 when unreadable)."""
        print(f"Generating detection JSON for {person_name}...")
        found = []
        for pattern in (f"{person_name}_face_*.jpg", "face_*_frame_*.jpg", "*.jpg"):
            for path in glob.glob(os.path.join(face_dir, pattern)):
                if not any(sk in os.path.basename(path).lower() for sk in _SKIP):
                    found.append(path)
        files = sorted(set(found))
        print(f"Found {len(files)} face images for {person_name}")
        if not files:
            print(f"No face images found for {person_name}")
            return None
        faces = []
        fps = 30.0
        for face_id, path in enumerate(files):
            name = os.path.basename(path)
            frame = 0
            m = re.search(r"face_\d+_frame_(\d+)", name)
            if m:
                frame = int(m.group(1))
            else:
                m = re.search(r"_face_(\d+)", name)
                if m:
                    frame = int(m.group(1))
            img = decode_image(path)
            h, w = (img.shape[0], img.shape[1]) if img is not None else (64, 64)
            faces.append({"face_id": face_id, "frame_number": frame, "timestamp": frame / fps, "x": 0, "y": 0,
                          "width": w, "height": h, "center_x": w // 2, "center_y": h // 2, "area": w * h,
                          "image_path": path, "image_filename": name})
        info = {"video_path": f"videos/{person_name}.mp4",
                "total_frames": max(f["frame_number"] for f in faces) + 1,
                "fps": fps, "total_faces_detected": len(faces),
                "processing_date": datetime.now().isoformat(), "faces": faces}
        json_path = os.path.join(face_dir, f"{person_name}_faces_detection.json")
        with open(json_path, "w", encoding="utf-8") as f:
            json.dump(info, f, indent=2, ensure_ascii=False)
        print(f"Generated {json_path}\nTotal faces: {len(faces)}")
        return json_path

    # --------------------------------------------------------------- counting
    def count_face_images_in_directory(self, directory):
        """train-v5.py:144-179: a base directory sums its person directories."""
        if not os.path.exists(directory):
            return 0
        subdirs = [d for d in os.listdir(directory) if os.path.isdir(os.path.join(directory, d))]
        if subdirs and any(os.path.exists(os.path.join(directory, d, f"{d}_faces_detection.json"))
                           or glob.glob(os.path.join(directory, d, "*.jpg")) for d in subdirs):
            total = 0
            for name in subdirs:
                cnt = self._count_face_images_in_single_dir(os.path.join(directory, name))
                total += cnt
                print(f"{name}: {cnt} face images")
            return total
        return self._count_face_images_in_single_dir(directory)

    def _count_face_images_in_single_dir(self, person_dir):
        """JPGs of the directory minus eigenface / mean_face / model_info images (:181-196)."""
        if not os.path.exists(person_dir):
            return 0
        return sum(1 for f in glob.glob(os.path.join(person_dir, "*.jpg"))
                   if not any(sk in os.path.basename(f).lower() for sk in _SKIP))

    # ---------------------------------------------------------------- loading
    def _load_rows(self, paths, infos):
        rows, keep = read_faces(paths, self.face_shape, self.device)  # one GPU grey+resize launch
        for i in sorted(set(range(len(paths))) - set(keep)):
            print(f"Warning: Could not read image {paths[i]}, skipping...")
        return rows, [infos[i] for i in keep]

    def load_all_face_images(self, base_dir):
        """Every person directory of base_dir with person ids in listing order
        (train-v5.py:198-274); a missing detection JSON is synthesised first."""
        print(f"Loading face data from all persons in {base_dir}")
        if not os.path.exists(base_dir):
            print(f"Error: Directory {base_dir} not found!")
            return 0
        person_dirs = [d for d in os.listdir(base_dir) if os.path.isdir(os.path.join(base_dir, d))]
        print(f"Found {len(person_dirs)} person directories: {person_dirs}")
        paths, infos = [], []
        pid = 0
        for name in person_dirs:
            pdir = os.path.join(base_dir, name)
            jp = os.path.join(pdir, f"{name}_faces_detection.json")
            if not os.path.exists(jp):
                print(f"JSON file not found for {name}, generating...")
                self.generate_detection_json_for_person(name, pdir)
            if not os.path.exists(jp):
                print(f"Warning: Could not generate JSON for {name}, skipping...")
                continue
            with open(jp, "r", encoding="utf-8") as f:
                faces = json.load(f)["faces"]
            print(f"Found {len(faces)} faces for {name}")
            self.person_id_map[name] = pid
            for info in faces:
                if not os.path.exists(info["image_path"]):
                    print(f"Warning: Image {info['image_path']} not found, skipping...")
                    continue
                info["person_name"] = name
                info["person_id"] = pid
                paths.append(info["image_path"])
                infos.append(info)
            pid += 1
        rows, self.face_info = self._load_rows(paths, infos)
        print(f"Successfully loaded {len(rows)} face images from {len(self.person_id_map)} persons")
        self.face_images = rows
        self.face_labels = np.array([i["person_id"] for i in self.face_info], dtype=np.int64)
        return len(rows)

    def load_face_images_from_json(self, json_path, person_dir):
        """One person's faces in JSON order (train-v5.py:276-347): ``image_filename``
        joined with person_dir first, else ``image_path``, else face_{id}_frame_{n}.jpg;
        labels all 0, person id map {dir name: 0}."""
        print(f"Loading face data from {json_path}")
        if not os.path.exists(json_path):
            print(f"Error: JSON file {json_path} not found!")
            return 0
        with open(json_path, "r", encoding="utf-8") as f:
            faces = json.load(f)["faces"]
        print(f"Found {len(faces)} faces in JSON")
        paths, infos = [], []
        for i, info in enumerate(faces):
            if "image_filename" in info:
                path = os.path.join(person_dir, info["image_filename"])
            elif "image_path" in info:
                path = info["image_path"]
            else:
                path = os.path.join(person_dir, f"face_{info.get('face_id', i)}_frame_{info.get('frame_number', i)}.jpg")
            if not os.path.exists(path):
                print(f"Warning: Image {path} not found, skipping...")
                continue
            paths.append(path)
            infos.append(info)
        rows, self.face_info = self._load_rows(paths, infos)
        print(f"Successfully loaded {len(rows)} face images")
        self.face_images = rows
        self.face_labels = np.zeros(len(rows), dtype=np.int64)
        self.person_id_map = {os.path.basename(os.path.normpath(person_dir)): 0}
        return len(rows)

    # ---------------------------------------------------------------- training
    def train_pca_model(self):
        """StandardScaler -> PCA(n_components) on the GPU (train-v5.py:349-385).  As with
        sklearn, n_components above min(n_samples, n_features) is an error (raised)."""
        if len(self.face_images) == 0:
            print("Error: No face images loaded!")
            return False
        if len(self.face_labels) == 0:
            print("Error: No face labels assigned!")
            return False
        n, d = self.face_images.shape
        print(f"\nTraining PCA model with {n} faces...")
        print(f"Original feature dimension: {d}")
        print(f"Reducing to {self.n_components} components")
        if not 0 < self.n_components <= min(n, d):  # sklearn _pca.py:_fit_full's check
            raise ValueError(f"n_components={self.n_components} must be between 0 and "
                             f"min(n_samples, n_features)={min(n, d)} with svd_solver='full'")
        try:
            m = EigenfacePCA(self.n_components, standardize=True, device=self.device).fit(self.face_images)
        except EigenfaceError as e:
            print(f"Error: PCA training failed: {e}")
            return False
        self.model = m
        self.mean_face = m.mean_face_
        self.scaler, self.pca = sklearn_objects(m)
        self.eigenfaces = self.pca.components_
        self.face_features = m.face_features_
        print(f"Mean face calculated with shape: {self.mean_face.shape}")
        print(f"Generated {len(self.eigenfaces)} eigenfaces")
        print(f"PCA explained variance ratio: {self.pca.explained_variance_ratio_.sum():.3f}")
        print(f"Reduced feature dimension: {self.face_features.shape[1]}")
        self.is_trained = True
        return True

    def save_eigenfaces(self, output_dir):
        """multi_person_mean_face.jpg, multi_person_eigenface_XX.jpg (top 10, min-max
        8-bit) and multi_person_model_info.json (train-v5.py:387-436)."""
        if not self.is_trained:
            print("Error: Model not trained yet!")
            return False
        os.makedirs(output_dir, exist_ok=True)
        _save_jpg(os.path.join(output_dir, "multi_person_mean_face.jpg"), self.mean_face.reshape(self.face_shape))
        n_save = min(10, len(self.eigenfaces))
        for i in range(n_save):
            _save_jpg(os.path.join(output_dir, f"multi_person_eigenface_{i + 1:02d}.jpg"),
                      self.eigenfaces[i].reshape(self.face_shape))
        info = {
            "training_date": datetime.now().isoformat(),
            "total_faces": len(self.face_images),
            "total_persons": len(self.person_id_map),
            "person_id_map": self.person_id_map,
            "n_components": self.n_components,
            "explained_variance_ratio": float(self.pca.explained_variance_ratio_.sum()),
            "face_shape": self.face_shape,
            "eigenfaces_saved": n_save,
        }
        with open(os.path.join(output_dir, "multi_person_model_info.json"), "w", encoding="utf-8") as f:
            json.dump(info, f, indent=2, ensure_ascii=False)
        return True

    def save_model(self, model_path):
        """face_model.pkl with the train-v4 key set (train-v5.py:438-467)."""
        if not self.is_trained:
            print("Error: Model not trained yet!")
            return False
        md = {"pca": self.pca, "scaler": self.scaler, "face_features": self.face_features,
              "face_labels": self.face_labels, "face_info": self.face_info, "person_id_map": self.person_id_map,
              "n_components": self.n_components, "mean_face": self.mean_face, "eigenfaces": self.eigenfaces,
              "face_shape": self.face_shape, "training_date": datetime.now().isoformat()}
        with open(model_path, "wb") as f:
            pickle.dump(md, f)
        print(f"Model saved to {model_path}")
        return True

    def load_model(self, model_path):
        """train-v5.py:469-505 (trusted files only: a pickle executes code on load)."""
        if not os.path.exists(model_path):
            print(f"Error: Model file {model_path} not found!")
            return False
        with open(model_path, "rb") as f:
            md = pickle.load(f)
        self.pca, self.scaler = md["pca"], md["scaler"]
        self.face_features, self.face_labels = md["face_features"], md["face_labels"]
        self.face_info, self.person_id_map = md["face_info"], md["person_id_map"]
        self.n_components = md["n_components"]
        self.mean_face = md.get("mean_face")
        self.eigenfaces = md.get("eigenfaces")
        self.face_shape = md.get("face_shape", (64, 64))
        self.is_trained = True
        return True


def train_person_model(person_name, base_dir, device=0):
    """train-v5.py:507-568: k = face count (full rank) for one person directory."""
    print(f"\n=== Training model for {person_name} ===")
    person_dir = os.path.join(base_dir, person_name)
    json_file = os.path.join(person_dir, f"{person_name}_faces_detection.json")
    model_path = os.path.join(person_dir, "face_model.pkl")
    if not os.path.exists(person_dir):
        print(f"Error: Person directory {person_dir} not found!")
        return False
    tmp = MultiFaceTrainer(device=device)
    face_count = tmp.count_face_images_in_directory(person_dir)
    if face_count == 0:
        print(f"No face images found for {person_name}!")
        return False
    if not os.path.exists(json_file):
        tmp.generate_detection_json_for_person(person_name, person_dir)
    k = face_count if face_count > 1 else 1
    print(f"Face images found for {person_name}: {face_count}")
    print(f"Setting n_components to: {k}")
    trainer = MultiFaceTrainer(n_components=k, device=device)
    if trainer.load_face_images_from_json(json_file, person_dir) == 0:
        print(f"No valid face images loaded for {person_name}!")
        return False
    if trainer.train_pca_model():
        trainer.save_eigenfaces(person_dir)
        trainer.save_model(model_path)
        print(f"Training completed successfully for {person_name}!")
        return True
    print(f"Training failed for {person_name}!")
    return False


def main(base_dir="faces/lock_version", device=0):
    """train-v5.py:570-610: train every person directory; returns (ok, failed)."""
    if not os.path.exists(base_dir):
        print(f"Error: Base directory {base_dir} not found!")
        return 0, 0
    person_dirs = [d for d in os.listdir(base_dir) if os.path.isdir(os.path.join(base_dir, d))]
    if not person_dirs:
        print(f"No person directories found in {base_dir}!")
        return 0, 0
    print(f"Found {len(person_dirs)} person directories: {person_dirs}")
    ok = failed = 0
    for name in person_dirs:
        try:
            if train_person_model(name, base_dir, device):
                ok += 1
            else:
                failed += 1
        except Exception as e:  # noqa: BLE001 - reference prints and counts (:594-601)
            print(f"Error training model for {name}: {e}")
            failed += 1
    print("\n=== Training Summary ===")
    print(f"Total persons processed: {len(person_dirs)}")
    print(f"Successful trainings: {ok}")
    print(f"Failed trainings: {failed}")
    return ok, failed

"""Drop-in for the reference's ``train-v4.py`` (what run_pipeline.py:234 runs as
``python train-v4.py --person P``): same command line, same inputs
(faces/lock_version/P/P_faces_detection.json + crops, relative to the working directory),
same outputs (faces/lock_version/P/face_model.pkl with real sklearn StandardScaler / PCA
objects, P_mean_face.jpg, P_eigenface_XX.jpg, P_model_info.json) and the same exit
status (0 after printing an error, as the reference's main returns), with the
StandardScaler + PCA fit on the GPU (libeigenface, gfx950).

Use: symlink or copy this file (and _locate.py) into a reference checkout, or run it in
place with the checkout as the working directory; set EIGENFACE_PKG to the
face-detection-recognization-pca_amd directory if the file was copied elsewhere.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.realpath(__file__)))
from _locate import locate  # noqa: E402

locate()
from eigenface.cli import main_train_v4  # noqa: E402

if __name__ == "__main__":
    main_train_v4()

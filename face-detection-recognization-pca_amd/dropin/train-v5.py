"""Drop-in for the reference's ``train-v5.py`` (no arguments): one model per directory
of faces/lock_version (n_components = the person's face count), detection JSONs
synthesised where missing, multi_person_* artefacts — the fit on the GPU
(eigenface.multi_person, train-v5.py:507-610)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.realpath(__file__)))
from _locate import locate  # noqa: E402

locate()
from eigenface.multi_person import main  # noqa: E402

if __name__ == "__main__":
    main()

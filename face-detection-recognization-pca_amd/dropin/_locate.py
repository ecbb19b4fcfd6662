"""Make the ``eigenface`` package importable for the drop-in scripts: the package
directory next to this file (the scripts are symlinked or run in place), else
$EIGENFACE_PKG, else an installed copy."""
import os
import sys


def locate():
    here = os.path.dirname(os.path.realpath(__file__))
    for cand in (os.path.dirname(here), os.environ.get("EIGENFACE_PKG", "")):
        if cand and os.path.isdir(os.path.join(cand, "eigenface")):
            if cand not in sys.path:
                sys.path.insert(0, cand)
            return cand
    return None

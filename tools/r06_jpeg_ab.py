"""A/B of the JPEG ingest stream with and without the early (phased) upload of the
destuffed words (EF_JPEG_EARLY_UP, read once per process: run once per setting)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "face-detection-recognization-pca_amd"))
import torch  # noqa: E402
import bench  # noqa: E402
from eigenface.engine import Engine  # noqa: E402

eng = Engine(0)
eng.timing(True)
sides = [s for grp in bench.TEMPLATE_SIDES for s in grp]
rows = []
for rep in range(3):
    r = bench.jpeg_ingest_bench(eng, False, sides, reps=20)
    r.pop("note", None)
    rows.append(r)
print(json.dumps({"early_up": os.environ.get("EF_JPEG_EARLY_UP", "1"), "runs": rows}))

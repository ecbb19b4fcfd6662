"""The oracle's restatement of the manual trainer's classes (scripts/manual/train-v2.py:
9-72) and the manual scanner's cosine (useless/scan.py:58-78) against the outputs of the
reference's own code (tests/golden/manual_v2.npz, make_goldens.py manual_v2)."""
import numpy as np
import pytest

from conftest import golden
from oracle import eigenface_oracle as orc


@pytest.mark.parametrize("tag", ["gram", "cov"])
def test_manual_trainer_oracle_matches_reference(tag):
    g = golden("manual_v2.npz")
    X = orc.int_synth_faces(int(g[f"{tag}_n"]), int(g[f"{tag}_side"]), r=int(g[f"{tag}_r"]),
                            seed=int(g[f"{tag}_seed"]))
    Z, mean, scale = orc.manual_standard_scaler(X)
    np.testing.assert_array_equal(mean, g[f"{tag}_scaler_mean"])
    np.testing.assert_array_equal(scale, g[f"{tag}_scaler_scale"])
    comps, _, evr, _, feats = orc.manual_pca_cov(Z, int(g[f"{tag}_k"]))
    np.testing.assert_allclose(comps, g[f"{tag}_components"], atol=1e-12)
    np.testing.assert_allclose(evr, g[f"{tag}_evr"], rtol=1e-12)
    np.testing.assert_allclose(feats, g[f"{tag}_features"], atol=1e-9)


def test_cosine_similarity_oracle_matches_reference():
    g = golden("manual_v2.npz")
    got = [orc.cosine_similarity_vec(a, b) for a, b in zip(g["cos_a"], g["cos_b"])]
    np.testing.assert_allclose(got, g["cos_sim"], rtol=1e-15, atol=1e-15)

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "consensus-entropy_amd")
for p in (ROOT, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")


def golden(name):
    import numpy as np

    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture
def load_golden():
    return golden


def fitted_members(seed=260, n_test=3000):
    """A GaussianNB and an SGDClassifier(log loss) fitted on synthetic 260-feature
    frames of 4 quadrant classes (the reference's member types, deam_classifier.py
    :211-218), plus held-out frames."""
    import numpy as np
    from sklearn.linear_model import SGDClassifier
    from sklearn.naive_bayes import GaussianNB

    rng = np.random.default_rng(seed)
    D, C = 260, 4
    centers = rng.normal(0, 1, (C, D))
    y = rng.integers(0, C, 4000)
    X = centers[y] + rng.normal(0, 2.0, (4000, D))
    gnb = GaussianNB().fit(X, y)
    sgd = SGDClassifier(loss="log_loss", penalty="l2", random_state=1987, max_iter=20, tol=None).fit(X, y)
    Xt = centers[rng.integers(0, C, n_test)] + rng.normal(0, 2.0, (n_test, D))
    return gnb, sgd, Xt

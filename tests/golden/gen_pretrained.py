"""Fixture generator: the reference's shipped committee members as plain arrays
(tests/golden/pretrained_members.npz), read by the no-code opcode walker
(pickle_walk.py: nothing in a pickle is imported, called or unpickled).

  models/pretrained/classifier_gnb.it_{0..4}.pkl  sklearn 0.24.1 GaussianNB:
      theta_ [4, 260], sigma_ [4, 260] (variance incl. epsilon_), class_prior_ [4]
  models/pretrained/classifier_sgd.it_{0..4}.pkl  SGDClassifier(loss='log'):
      coef_ [4, 260], intercept_ [4]
  models/pretrained/classifier_xgb.it_{0..4}.pkl  XGBClassifier (xgboost 1.3.3):
      the booster's serialised JSON 'Model' (the save_model schema; 400 trees,
      multi:softprob, 4 classes), stored as UTF-8 bytes

These are the member files amg_test.py copies per user (:347-351, os.walk
order) and calls predict_proba on (:435).  Run in this container only (the
reference does not travel):  python tests/golden/gen_pretrained.py [REF_ROOT]
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import pickle_walk as W  # noqa: E402


def extract(ref_root="/root/reference"):
    d = os.path.join(ref_root, "models", "pretrained")
    out = {}
    src = {}
    g = [W.read_gnb(open(os.path.join(d, f"classifier_gnb.it_{k}.pkl"), "rb").read()) for k in range(5)]
    s = [W.read_sgd(open(os.path.join(d, f"classifier_sgd.it_{k}.pkl"), "rb").read()) for k in range(5)]
    out["gnb_theta"] = np.stack([m["theta"] for m in g])
    out["gnb_var"] = np.stack([m["var"] for m in g])
    out["gnb_prior"] = np.stack([m["class_prior"] for m in g])
    out["gnb_classes"] = np.stack([m["classes"] for m in g])
    out["sgd_coef"] = np.stack([m["coef"] for m in s])
    out["sgd_intercept"] = np.stack([m["intercept"] for m in s])
    out["sgd_classes"] = np.stack([m["classes"] for m in s])
    assert all(m["loss"] == "log" for m in s)
    for k in range(5):
        x = W.read_xgb(open(os.path.join(d, f"classifier_xgb.it_{k}.pkl"), "rb").read())
        out[f"xgb_model_{k}"] = np.frombuffer(json.dumps(x["model"], separators=(",", ":")).encode(), np.uint8)
    for fn in sorted(os.listdir(d)):
        if fn.endswith(".pkl"):
            src[fn] = hashlib.sha256(open(os.path.join(d, fn), "rb").read()).hexdigest()
    out["source_sha256"] = np.frombuffer(json.dumps(src, sort_keys=True).encode(), np.uint8)
    return out


if __name__ == "__main__":
    arrs = extract(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
    np.savez_compressed(os.path.join(HERE, "pretrained_members.npz"), **arrs)
    print({k: v.shape for k, v in arrs.items()})

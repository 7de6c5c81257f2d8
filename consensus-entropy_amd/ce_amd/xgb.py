"""XGBoost forests for the on-device 'classifier_xgb' committee member
(amg_test.py:435/:467 -> xgboost/sklearn.py:991-1029).

The reference's member is ``XGBClassifier(max_depth=5, ...)`` from xgboost
1.3.3 (deam_classifier.py:226-232, requirements.txt:50), read back from
pickles.  Pickles are never loaded here; a forest comes from xgboost's own
JSON model format -- ``booster.save_model("m.json")`` (or ``save_raw`` in
later versions) -- whose schema this module parses:

    learner.learner_model_param.{base_score, num_class, num_feature}
    learner.objective.name                       multi:softprob | binary:logistic
    learner.gradient_booster.model.tree_info     group of tree t
    learner.gradient_booster.model.trees[t].{left_children, right_children,
        split_indices, split_conditions (the leaf value at a leaf), default_left}

``XgbForest.pack`` turns it into the device layout of ce_xgb_predict_proba:
perfect trees of the forest's depth, group-major.  ``synthetic_model`` makes a
random forest in that JSON schema (bench / tests: there is no network to fetch
a trained model, and the reference's pickles are untrusted).
"""
from __future__ import annotations

import ctypes
import ctypes.util
import json
import os

import numpy as np

MAX_DEPTH = 10
MAX_FEATURES = 512
MAX_GROUPS = 8

_libm = None


def _logf(x):
    """libm's logf (xgboost's ProbToMargin runs in float32 through it)."""
    global _libm
    if _libm is None:
        _libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
        _libm.logf.restype = ctypes.c_float
        _libm.logf.argtypes = [ctypes.c_float]
    return np.float32(_libm.logf(ctypes.c_float(x)))


class XgbForest:
    """A parsed xgboost 1.3 model: per-tree node arrays in model order."""

    def __init__(self, trees, tree_info, num_class, base_score, objective, num_feature):
        self.trees = trees                  # list of dicts of numpy arrays
        self.tree_info = np.asarray(tree_info, dtype=np.int32)
        self.num_class = int(num_class)     # 0 or 1 for binary:logistic (xgboost's convention)
        self.base_score = np.float32(base_score)
        self.objective = objective
        self.num_feature = int(num_feature)
        self._packed = None
        self._dev = {}

    # ---- construction -------------------------------------------------------
    @classmethod
    def from_json(cls, model):
        """``model``: a dict, a JSON string, or a path to ``booster.save_model(*.json)``."""
        if isinstance(model, (str, bytes, os.PathLike)):
            if isinstance(model, (str, os.PathLike)) and os.path.exists(model):
                with open(model) as fh:
                    model = json.load(fh)
            else:
                model = json.loads(model)
        lrn = model["learner"]
        mp = lrn["learner_model_param"]
        objective = lrn.get("objective", {}).get("name", "multi:softprob")
        if objective not in ("multi:softprob", "binary:logistic"):
            # multi:softmax's booster output is the class label; XGBClassifier.predict_proba
            # then returns [1 - label, label] (xgboost/sklearn.py:1025-1029), not probabilities
            raise ValueError(f"objective {objective!r} has no probability output (multi:softprob or "
                             "binary:logistic only)")
        gb = lrn["gradient_booster"]
        if gb.get("name", "gbtree") != "gbtree":
            raise ValueError(f"booster {gb.get('name')!r} unsupported (gbtree only)")
        m = gb["model"]
        trees = []
        for t in m["trees"]:
            tr = {
                "left": np.asarray(t["left_children"], dtype=np.int32),
                "right": np.asarray(t["right_children"], dtype=np.int32),
                "split": np.asarray(t["split_indices"], dtype=np.int32),
                "cond": np.asarray(t["split_conditions"], dtype=np.float32),
                "default_left": np.asarray([bool(v) for v in t["default_left"]], dtype=np.uint8),
            }
            n = tr["left"].size
            if not all(a.size == n for a in tr.values()) or n == 0:
                raise ValueError("inconsistent tree node arrays")
            trees.append(tr)
        return cls(trees, m["tree_info"], int(mp.get("num_class", "0")), float(mp["base_score"]), objective,
                   int(mp.get("num_feature", "0")))

    @classmethod
    def from_booster(cls, booster):  # pragma: no cover - xgboost is not installed in this image
        """From a live ``xgboost.Booster`` (or XGBClassifier): its JSON model."""
        import tempfile

        booster = booster.get_booster() if hasattr(booster, "get_booster") else booster
        with tempfile.TemporaryDirectory() as d:
            path = os.path.join(d, "model.json")
            booster.save_model(path)
            return cls.from_json(path)

    # ---- derived geometry ---------------------------------------------------
    @property
    def n_groups(self):
        return 1 if self.objective == "binary:logistic" else self.num_class

    @property
    def n_classes(self):
        return 2 if self.objective == "binary:logistic" else self.num_class

    @property
    def base_margin(self):
        """xgboost's LearnerModelParam base margin: ProbToMargin(base_score)."""
        if self.objective == "binary:logistic":
            b = self.base_score
            return np.float32(-_logf(np.float32(np.float32(1.0) / b - np.float32(1.0))))
        return self.base_score

    def depth(self):
        d = 0
        for tr in self.trees:
            stack = [(0, 0)]
            while stack:
                nid, dep = stack.pop()
                if tr["left"][nid] == -1:
                    d = max(d, dep)
                else:
                    stack.append((int(tr["left"][nid]), dep + 1))
                    stack.append((int(tr["right"][nid]), dep + 1))
        return d

    # ---- the device layout --------------------------------------------------
    def pack(self):
        """(nodes u32 [T, 2^d - 1, 2], leaves f32 [T, 2^d], group_offsets i32 [G+1], depth):
        perfect trees, group-major, model order inside a group."""
        if self._packed is not None:
            return self._packed
        G = self.n_groups
        if G < 1 or G > MAX_GROUPS:
            raise ValueError(f"{G} groups: 1..{MAX_GROUPS} supported")
        if self.tree_info.size != len(self.trees) or (self.tree_info.size and (
                self.tree_info.min() < 0 or self.tree_info.max() >= G)):
            raise ValueError("tree_info does not match the trees / groups")
        d = self.depth()
        if d > MAX_DEPTH:
            raise ValueError(f"tree depth {d} > {MAX_DEPTH}")
        NI, NL = (1 << d) - 1, 1 << d
        order = np.argsort(self.tree_info, kind="stable")  # group-major, model order kept
        T = len(self.trees)
        nodes = np.zeros((T, max(NI, 1), 2), dtype=np.uint32)
        leaves = np.zeros((T, NL), dtype=np.float32)
        for k, t in enumerate(order):
            tr = self.trees[t]
            # walk the model tree alongside the perfect tree: (model node, perfect index, depth)
            stack = [(0, 0, 0)]
            while stack:
                nid, pi, dep = stack.pop()
                if tr["left"][nid] == -1:
                    # a leaf at depth dep covers perfect leaves [lo, lo + 2^(d-dep))
                    lo = ((pi + 1) << (d - dep)) - 1 - NI
                    leaves[k, lo:lo + (1 << (d - dep))] = tr["cond"][nid]
                    continue  # internal nodes below it stay {0, +0.0}: either branch, same leaf
                f = int(tr["split"][nid])
                if f < 0 or f >= MAX_FEATURES or (self.num_feature and f >= self.num_feature):
                    raise ValueError(f"split feature {f} out of range")
                nodes[k, pi, 0] = np.uint32(f) | (np.uint32(1 << 31) if tr["default_left"][nid] else np.uint32(0))
                nodes[k, pi, 1] = np.float32(tr["cond"][nid]).view(np.uint32)
                stack.append((int(tr["left"][nid]), 2 * pi + 1, dep + 1))
                stack.append((int(tr["right"][nid]), 2 * pi + 2, dep + 1))
        counts = np.bincount(self.tree_info, minlength=G)
        goff = np.zeros(G + 1, dtype=np.int32)
        goff[1:] = np.cumsum(counts)
        self._packed = (nodes, leaves, goff, d)
        return self._packed

    def max_feature(self):
        return max((int(tr["split"][tr["left"] != -1].max(initial=-1)) for tr in self.trees), default=-1)

    def lane_table(self, device, D):
        """The prebuilt per-tree lane tables of ce_xgb_predict_proba_lanes (depth
        <= 5): int32 [2, T, 64, 2] on ``device`` for X with D columns (with and
        without the default-left bits), built once on the device by
        ce_xgb_lane_table and cached per (device, D)."""
        import torch

        from . import _lib
        from .ops import _p, _stream, call

        key = (torch.device(device), int(D))
        if key not in self._dev:
            nodes, leaves, _, d = self.device_arrays(device)
            T = len(self.trees)
            table = torch.empty((2, T, 64, 2), dtype=torch.int32, device=key[0])
            _lib.load()
            call("ce_xgb_lane_table", _p(nodes), _p(leaves), T, d, int(D), _p(table), _stream(key[0]))
            self._dev[key] = table
        return self._dev[key]

    def device_arrays(self, device):
        """The packed arrays as device tensors (cached per device)."""
        import torch

        key = torch.device(device)
        if key not in self._dev:
            nodes, leaves, goff, d = self.pack()
            self._dev[key] = (torch.from_numpy(nodes.view(np.int32)).to(key),
                              torch.from_numpy(leaves).to(key), torch.from_numpy(goff).to(key), d)
        return self._dev[key]


def synthetic_model(n_rounds=100, num_class=4, max_depth=5, num_feature=260, seed=1987, p_stop=0.15,
                    objective=None, threshold_scale=1.0):
    """A random xgboost-1.3-JSON forest: ``n_rounds`` boosting rounds x groups
    trees (tree t of round r belongs to group t % groups, as xgboost grows
    them), node ids allocated in expansion order, early leaves with
    probability ``p_stop`` per internal node below the root, thresholds and
    leaf weights float32, random default directions.  The reference's member
    is XGBClassifier(max_depth=5) on 260 standardised features, 4 classes."""
    rng = np.random.default_rng(seed)
    if objective is None:
        objective = "binary:logistic" if num_class <= 2 else "multi:softprob"
    groups = 1 if objective == "binary:logistic" else num_class
    trees, tree_info = [], []
    for r in range(n_rounds):
        for g in range(groups):
            left, right, split, cond, dflt = [], [], [], [], []

            def new_node():
                left.append(-1)
                right.append(-1)
                split.append(0)
                cond.append(0.0)
                dflt.append(0)
                return len(left) - 1

            root = new_node()
            frontier = [(root, 0)]
            while frontier:  # breadth-first, like xgboost's depthwise grower
                nxt = []
                for nid, dep in frontier:
                    leaf = dep >= max_depth or (dep > 0 and rng.random() < p_stop)
                    if leaf:
                        cond[nid] = float(np.float32(rng.normal(0.0, 0.2)))
                        continue
                    split[nid] = int(rng.integers(0, num_feature))
                    cond[nid] = float(np.float32(rng.normal(0.0, threshold_scale)))
                    dflt[nid] = int(rng.integers(0, 2))
                    lc, rc = new_node(), new_node()
                    left[nid], right[nid] = lc, rc
                    nxt += [(lc, dep + 1), (rc, dep + 1)]
                frontier = nxt
            n = len(left)
            trees.append({"tree_param": {"num_nodes": str(n), "num_feature": str(num_feature),
                                         "size_leaf_vector": "0", "num_deleted": "0"},
                          "id": len(trees), "left_children": left, "right_children": right,
                          "parents": [2147483647] + [0] * (n - 1), "split_indices": split,
                          "split_conditions": cond, "default_left": [bool(v) for v in dflt],
                          "loss_changes": [0.0] * n, "sum_hessian": [1.0] * n, "base_weights": [0.0] * n})
            tree_info.append(g)
    return {"learner": {
        "learner_model_param": {"base_score": "5E-1", "num_class": str(num_class if groups > 1 else 0),
                                "num_feature": str(num_feature)},
        "objective": {"name": objective},
        "gradient_booster": {"name": "gbtree", "model": {
            "gbtree_model_param": {"num_trees": str(len(trees)), "size_leaf_vector": "0"},
            "trees": trees, "tree_info": tree_info}},
        "attributes": {}, "feature_names": [], "feature_types": []},
        "version": [1, 3, 3]}

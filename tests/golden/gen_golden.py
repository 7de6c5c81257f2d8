"""Generate the golden fixtures for the selection path.

Runs the reference's own expressions VERBATIM with numpy/scipy in this
container (oracle/ce_oracle.py ``ref_*``: amg_test.py:441-445, :451-452,
:473-480, :69-78, :109-117) on seeded synthetic inputs (seed 1987, the
reference's seed at amg_test.py:55) and writes the inputs and outputs as small
.npz files next to this script.  The reference module itself cannot be imported
here (ordinary ImportErrors: tensorboard / torchaudio / xgboost absent), but the
path's arithmetic lives in numpy/scipy, which are importable -- so these
expressions ARE the reference's computation.

Also records the paper's worked examples (ISMIR2021 p.3 sec.3.2).

Usage:  python tests/golden/gen_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle.ce_oracle import (canonical_order, ref_hc, ref_mc, ref_mix,  # noqa: E402
                              ref_quadrant, ref_vote_table)

SEED = 1987
Q = 10


def dirichlet(rng, shape):
    e = -np.log(rng.random(shape))
    return e / e.sum(axis=-1, keepdims=True)


def to_bf16_exact(x):
    """Round f32 values to the nearest bf16 and return (f32 values, uint16 bits)."""
    u = np.asarray(x, dtype=np.float32).view(np.uint32)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    return (r.astype(np.uint32) << 16).view(np.float32), r


def save(name, **arrs):
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrs)
    print(f"{name}: " + ", ".join(f"{k}{tuple(v.shape)}" for k, v in arrs.items()))


def mc_case(name, pred_prob, q=Q):
    stack = np.array(pred_prob)  # what amg_test.py:441 builds
    q_ind, ent, mean = ref_mc(pred_prob, q)
    save(name, P=stack, ent=ent, mean=mean, q_ind=np.asarray(q_ind, np.int64),
         canon=canonical_order(ent, q), q=np.int64(q))


def main():
    rng = np.random.default_rng(SEED)

    # --- paper worked examples (p.3 sec.3.2) -------------------------------
    full = [np.eye(4)[[k]] for k in range(4)]            # 4 members, 100% each on a different quadrant
    _, ent_full, _ = ref_mc(full, 1)
    six = np.array([[0, 1, 1, 2, 2, 2]], dtype=np.int8)  # 6 annotators, counts {1,2,3,0}
    freq_six = ref_vote_table(six)
    _, ent_six = ref_hc(freq_six, 1)
    _, ent_unan = ref_hc(np.array([[1.0, 0.0, 0.0, 0.0]]), 1)
    save("paper_examples", ent_full=ent_full, freq_six=freq_six, ent_six=ent_six,
         ent_unanimous=ent_unan)

    # --- C1: mc, 4-member committee (gnb,sgd f64; xgb,cnn f32) x 1608 x 4 --
    N = 1608
    members = [dirichlet(rng, (N, 4)), dirichlet(rng, (N, 4)),
               dirichlet(rng, (N, 4)).astype(np.float32),
               dirichlet(rng, (N, 4)).astype(np.float32)]
    mc_case("mc_m4_mixed", members)

    # --- the paper's 20-member committee; 5 CNN members are sigmoid outputs
    #     (short_cnn.py:347, rows do not sum to 1) ------------------------------
    members = []
    for _ in range(5):
        members.append(dirichlet(rng, (N, 4)))                           # gnb
    for _ in range(5):
        members.append(dirichlet(rng, (N, 4)))                           # sgd
    for _ in range(5):
        members.append(dirichlet(rng, (N, 4)).astype(np.float32))        # xgb
    for _ in range(5):
        z = rng.normal(size=(N, 4))
        members.append((1.0 / (1.0 + np.exp(-z))).astype(np.float32))   # cnn sigmoid
    mc_case("mc_m20_mixed_unnorm", members)

    # --- all-fp32 16-member committee: engine contract = fp64 accumulate, so
    #     the reference expression runs on the fp64 upcast --------------------
    P32 = dirichlet(rng, (16, 4096, 4)).astype(np.float32)
    P32[:, ::97, :] *= np.float32(1.7)  # ~1% un-normalized rows
    mc_case("mc_m16_f32", list(P32.astype(np.float64)))

    # --- bf16-representable committee ---------------------------------------
    vals, bits = to_bf16_exact(dirichlet(rng, (8, 2048, 4)))
    q_ind, ent, mean = ref_mc(list(vals.astype(np.float64)), Q)
    save("mc_m8_bf16", P_bits=bits, P=vals.astype(np.float64), ent=ent,
         q_ind=np.asarray(q_ind, np.int64), canon=canonical_order(ent, Q), q=np.int64(Q))

    # --- tie-heavy: probabilities quantized to 1/8 ---------------------------
    Pq = np.floor(dirichlet(rng, (4, 3000, 4)) * 8) / 8.0
    Pq[..., 0] += 1.0 - Pq.sum(axis=-1)  # keep rows summing to 1, all k/8
    mc_case("mc_ties_q8", list(Pq), q=50)

    # --- NaN / zero rows / negatives / -0.0 / one-hot rows -------------------
    Pe = dirichlet(rng, (4, 512, 4))
    Pe[:, 7, :] = 0.0                      # zero row -> 0/0 -> NaN (ranked first)
    Pe[:, 100, :] = 0.0
    Pe[2, 33, 1] = -0.05                   # negative -> entr=-inf (ranked last)
    Pe[:, 40, :] = np.eye(4)[1]            # unanimous one-hot -> 0.0
    Pe[:, 41, :] = np.eye(4)[2]
    Pe[:, 42, :] = -0.0
    Pe[:, 42, 3] = 1.0                     # -0.0 entries
    Pe[1, 300, 2] = np.nan                 # NaN input propagates
    mc_case("mc_edge_nan_zero", list(Pe), q=12)

    # --- wide class counts: numpy pairwise summation order --------------------
    for C in (8, 9, 16, 100, 129, 1000):
        Pw = dirichlet(rng, (3, 64, C))
        Pw[0] *= 1.3
        mc_case(f"mc_wide_c{C}", list(Pw), q=8)

    # --- C2: hc votes [1608, 665] int8, 3% and 100% density ------------------
    for dens, tag in ((0.03, "d03"), (1.0, "d100")):
        votes = rng.integers(0, 4, size=(1608, 665)).astype(np.int8)
        miss = rng.random((1608, 665)) >= dens
        votes[miss] = -1
        votes[miss.all(axis=1), 0] = 1     # every song has >= 1 vote (as in :101-110)
        freq = ref_vote_table(votes)
        q_ind, ent = ref_hc(freq, Q)
        save(f"hc_votes_{tag}", votes=votes, freq=freq, ent=ent,
             q_ind=np.asarray(q_ind, np.int64), canon=canonical_order(ent, Q), q=np.int64(Q))

    # --- C2: mix = [mc mean; hc table] row stack ------------------------------
    members = [dirichlet(rng, (N, 4)), dirichlet(rng, (N, 4)),
               dirichlet(rng, (N, 4)).astype(np.float32),
               dirichlet(rng, (N, 4)).astype(np.float32)]
    votes = rng.integers(0, 4, size=(1300, 40)).astype(np.int8)
    votes[rng.random((1300, 40)) < 0.5] = -1
    votes[:, 0] = rng.integers(0, 4, size=1300)
    hc = ref_vote_table(votes)
    q_ind, ent = ref_mix(members, hc, Q)
    save("mix_m4", P=np.array(members), hc=hc, ent=ent, q_ind=np.asarray(q_ind, np.int64),
         canon=canonical_order(ent, Q), q=np.int64(Q))

    # --- raw valence/arousal -> quadrant -> frequencies (amg_test.py:93-117) --
    Nv, A = 300, 60
    va = rng.uniform(-1, 1, size=(Nv, A, 2))
    va[rng.random((Nv, A)) < 0.4] = np.nan          # missing annotations
    va[:, :3, :] = rng.uniform(-1, 1, size=(Nv, 3, 2))
    va[5, 3:9] = [[0.0, 0.3], [0.0, -0.3], [0.3, 0.0], [-0.3, 0.0], [0.0, 0.0], [-0.0, -0.0]]
    va[6, 3, 0] = np.nan                            # only one coordinate missing
    quad = np.full((Nv, A), -1, dtype=np.int8)
    for n in range(Nv):
        for a in range(A):
            v, ar = va[n, a]
            if np.isnan(v) or np.isnan(ar):
                continue  # dropna() at amg_test.py:101
            quad[n, a] = int(ref_quadrant(ar, v)[1]) - 1
    freq = ref_vote_table(quad)
    q_ind, ent = ref_hc(freq, Q)
    save("hc_va_raw", va=va, quad=quad, freq=freq, ent=ent,
         q_ind=np.asarray(q_ind, np.int64), canon=canonical_order(ent, Q), q=np.int64(Q))

    # --- C3: batched users, ragged pools --------------------------------------
    U = 8
    sizes = rng.integers(128, 1609, size=U)
    sizes[0] = 3          # pool smaller than q
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    Pb = dirichlet(rng, (4, int(offs[-1]), 4)).astype(np.float32)
    ents, canons = [], []
    for u in range(U):
        seg = Pb[:, offs[u]:offs[u + 1], :].astype(np.float64)
        q_ind, ent, _ = ref_mc(list(seg), Q)
        ents.append(ent)
        c = np.full(Q, -1, np.int64)
        cc = canonical_order(ent, Q)
        c[:len(cc)] = cc
        canons.append(c)
    save("batched_u8", P=Pb, offsets=offs, ent=np.concatenate(ents), canon=np.stack(canons),
         q=np.int64(Q))


if __name__ == "__main__":
    main()

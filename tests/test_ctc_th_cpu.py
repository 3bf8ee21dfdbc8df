"""CPU pin of the CTCPrefixScoreTH golden (tests/golden/ctc_th.npz, captured from the reference):
the numpy CTCPrefixScore restatement (oracle/asr_oracle.py OracleCTCPrefixScore, ctc_prefix_score.py:
272-358) run per utterance on its own frames only, with TH's bookkeeping (<eos> always scored,
blank and unscored labels logzero, scoring_idmap fallback to candidate 0), reproduces every
step's scores — the premise of the device implementation (espnet_amd/asr/ctc_prefix_score.py),
which also visits each utterance's own frames only."""
import numpy as np

from goldens import load
from oracle.asr_oracle import OracleCTCPrefixScore

LOGZERO = -10000000000.0


def test_ctc_th_golden_equals_per_utterance_numpy_restatement():
    cfg, d = load("ctc_th")
    B, O, W, eos, blank = cfg["B"], cfg["O"], cfg["W"], cfg["eos"], cfg["blank"]
    x, xlens = d["x"], d["xlens"]
    ora = [OracleCTCPrefixScore(x[b, :xlens[b]], blank, eos) for b in range(B)]
    n_bh = B * W
    r_prev = [ora[i // W].initial_state() for i in range(n_bh)]
    s_prev = np.zeros((n_bh, 1), dtype=np.float32)
    step = 0
    while f"s{step}.scores" in d:
        y = d[f"s{step}.y"]
        ids = d.get(f"s{step}.ids")
        log_psi = np.full((n_bh, O), LOGZERO, dtype=np.float32)
        r_new, cands = [], []
        for i in range(n_bh):
            cs = np.arange(O) if ids is None else ids[i]
            psi, rr = ora[i // W](list(y[i]), np.asarray(cs), r_prev[i])
            log_psi[i, cs] = psi
            log_psi[i, eos] = np.logaddexp(r_prev[i][-1, 0], r_prev[i][-1, 1])  # TH: always
            r_new.append(rr)
            cands.append(list(cs))
        log_psi[:, blank] = LOGZERO
        mine = log_psi - s_prev
        ref = d[f"s{step}.scores"]
        low = ref < -1e9
        assert np.array_equal(mine < -1e9, low), step
        np.testing.assert_allclose(mine[~low], ref[~low], rtol=1e-5, atol=2e-4, err_msg=f"step {step}")
        if f"s{step}.best" not in d:
            break
        best = d[f"s{step}.best"]
        nr, ns = [], []
        for b in range(B):
            for w in range(W):
                h, lab = divmod(int(best[b, w]), O)
                gh = b * W + h
                pos = cands[gh].index(lab) if lab in cands[gh] else 0
                nr.append(r_new[gh][pos])
                ns.append(log_psi[gh, lab])
        r_prev, s_prev = nr, np.asarray(ns, dtype=np.float32).reshape(-1, 1)
        step += 1
    assert step == 2

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


def _window(att_w, T, margin, ol, fmin_prev, fmax_prev):
    """ctc_prefix_score.py:144-149: the frames [start, end) around the attended frames."""
    f_arg = att_w.astype(np.float32) @ np.arange(T, dtype=np.float32)
    f_min = max(int(f_arg.min()), fmin_prev)
    f_max = max(int(f_arg.max()), fmax_prev)
    return min(fmax_prev, max(f_min - margin, ol, 1)), min(f_max + margin, T), f_min, f_max


def _th_steps(d, pre, B, W, O, eos, blank, ora_for, window_for=None, before=None):
    """Drive the per-utterance numpy restatement through the golden's steps with TH's
    bookkeeping; returns the number of selections made."""
    n_bh = B * W
    r_prev = [ora_for(i // W, 0).initial_state() for i in range(n_bh)]
    s_prev = np.zeros((n_bh, 1), dtype=np.float32)
    fm = (0, 1)
    step = 0
    while f"{pre}s{step}.scores" in d:
        if before is not None:
            r_prev = before(step, r_prev)
        y = d[f"{pre}s{step}.y"]
        ids = d.get(f"{pre}s{step}.ids")
        win = None
        if window_for is not None:
            start, end, fmin, fmax = window_for(step, len(y[0]) - 1, *fm)
            assert [fmin, fmax] == d[f"{pre}s{step}.fminmax"].tolist(), step
            win, fm = (start, end), (fmin, fmax)
        log_psi = np.full((n_bh, O), LOGZERO, dtype=np.float32)
        r_new, cands = [], []
        for i in range(n_bh):
            cs = np.arange(O) if ids is None else ids[i]
            psi, rr = ora_for(i // W, step)(list(y[i]), np.asarray(cs), r_prev[i], window=win)
            log_psi[i, cs] = psi
            log_psi[i, eos] = np.logaddexp(r_prev[i][-1, 0], r_prev[i][-1, 1])
            r_new.append(rr)
            cands.append(list(cs))
        log_psi[:, blank] = LOGZERO
        mine = log_psi - s_prev
        ref = d[f"{pre}s{step}.scores"]
        low = ref < -1e9
        assert np.array_equal(mine < -1e9, low), step
        np.testing.assert_allclose(mine[~low], ref[~low], rtol=1e-5, atol=2e-4, err_msg=f"{pre} step {step}")
        if f"{pre}s{step}.best" not in d:
            break
        best = d[f"{pre}s{step}.best"]
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
    return step


def test_ctc_th_window_and_streaming_golden_equal_numpy_restatement():
    """tests/golden/ctc_th_ext.npz (the reference's CTCPrefixScoreTH with margin 3 and attention
    weights; and its extend_prob / extend_state over 12 -> 20 -> 30 frames) against the
    restatement with the window's frame range and the blank-recursion state extension."""
    cfg, d = load("ctc_th_ext")
    O, W, eos, blank, margin = cfg["O"], cfg["W"], cfg["eos"], cfg["blank"], cfg["margin"]
    x, xlens = d["w.x"], d["w.xlens"]
    B, T = x.shape[0], x.shape[1]
    ora = [OracleCTCPrefixScore(x[b, :xlens[b]], blank, eos) for b in range(B)]
    n = _th_steps(d, "w.", B, W, O, eos, blank, lambda b, s: ora[b],
                  window_for=lambda s, ol, a, b: _window(d[f"w.s{s}.att_w"], T, margin, ol, a, b))
    assert n == 2
    xs, chunks = d["s.x"][0], cfg["chunks"]
    oras = [OracleCTCPrefixScore(xs[:c], blank, eos) for c in chunks]
    n = _th_steps(d, "s.", 1, W, O, eos, blank, lambda b, s: oras[s],
                  before=lambda s, rp: rp if s == 0 else [oras[s].extend_state(r) for r in rp])
    assert n == 2

"""Joint CTC/attention beam search on the C3 model (Conformer-L + 6-layer Transformer decoder,
V=5000, random init): one 1000-frame utterance (249 encoder frames), beam 10, ctc_weight 0.3,
a fixed 40-token output (maxlenratio -40, the C3 label length).  Prints the decode time per
utterance (and with --split the time in decoder scoring / CTC prefix scoring, measured with
synchronisations that themselves add to the total).

    python scripts/decode_bench.py [--beam 10] [--ctc-weight 0.3] [--tokens 40] [--utts 3]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "espnet-1_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--beam", type=int, default=10)
    ap.add_argument("--ctc-weight", type=float, default=0.3)
    ap.add_argument("--tokens", type=int, default=40)
    ap.add_argument("--utts", type=int, default=3)
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--single", action="store_true", help="BeamSearch (per-hypothesis selection on the host) "
                    "instead of BatchBeamSearch, the reference's default for batch scorers")
    ap.add_argument("--host-select", action="store_true", help="BatchBeamSearch with the host selection")
    ap.add_argument("--split", action="store_true", help="synchronise around the decoder / CTC scoring calls to "
                    "report their time (the syncs themselves add to the total)")
    ap.add_argument("--cprofile", action="store_true", help="host profile of the timed decodes (top 30)")
    args = ap.parse_args()
    from espnet_amd.asr.beam_search import BatchBeamSearch, BeamSearch, CTCPrefixScorer, LengthBonus
    dev = torch.device("cuda", 0)
    cfg = bench.c3_config()
    model = bench.build(cfg)
    model.prepare(dev, amp=not args.fp32, seed=1)
    model.eval()
    V = model.vocab_size
    timers = {"decoder": 0.0, "ctc": 0.0}

    def timed(name, fn):
        if not args.split:
            return fn

        def wrap(*a, **k):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = fn(*a, **k)
            torch.cuda.synchronize()
            timers[name] += time.perf_counter() - t0
            return out
        return wrap

    ctc = CTCPrefixScorer(model.ctc, model.eos)
    ctc.score_partial_multi = timed("ctc", ctc.score_partial_multi)  # host-selection paths only
    dec = model.decoder
    dec_batch_score = dec.batch_score
    dec.batch_score = timed("decoder", dec_batch_score)
    if args.host_select:
        BatchBeamSearch.device_select = False
    cls = BeamSearch if args.single else BatchBeamSearch
    bs = cls(scorers={"decoder": dec, "ctc": ctc, "length_bonus": LengthBonus(V)},
                    weights={"decoder": 1.0 - args.ctc_weight, "ctc": args.ctc_weight, "length_bonus": 0.0},
                    beam_size=args.beam, vocab_size=V, sos=model.sos, eos=model.eos, pre_beam_score_key="full")
    g = torch.Generator().manual_seed(3)
    speech = torch.randn(1, cfg["T"], cfg["input_size"], generator=g).to(dev)
    lens = torch.tensor([cfg["T"]], device=dev)
    with torch.no_grad():
        enc, _ = model.encode(speech, lens)  # warm-up (kernels, allocator)
        bs(enc[0], maxlenratio=-2)
        torch.cuda.synchronize()
        timers.update(decoder=0.0, ctc=0.0)
        t_enc = 0.0
        prof = None
        if args.cprofile:
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        t0 = time.perf_counter()
        for _ in range(args.utts):
            te = time.perf_counter()
            enc, _ = model.encode(speech, lens)
            torch.cuda.synchronize()
            t_enc += time.perf_counter() - te
            nbest = bs(enc[0], maxlenratio=-float(args.tokens))
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if prof is not None:
            import pstats
            prof.disable()
            pstats.Stats(prof).sort_stats("tottime").print_stats(30)
    n = args.utts
    print(f"C3 joint decode ({cls.__name__}{', host selection' if args.host_select else ''}): beam {args.beam}, ctc_weight {args.ctc_weight}, {args.tokens} tokens, "
          f"T'={enc.shape[1]}: {el / n * 1e3:.1f} ms/utt ({n / el:.2f} utt/s); encode {t_enc / n * 1e3:.1f} ms"
          + (f", decoder scoring {timers['decoder'] / n * 1e3:.1f} ms, CTC prefix scoring "
             f"{timers['ctc'] / n * 1e3:.1f} ms per utt (synchronised split)" if args.split else "")
          + f"; best hyp len {len(nbest[0].yseq) - 2}", flush=True)


if __name__ == "__main__":
    main()

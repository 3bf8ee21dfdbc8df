"""Per-tensor gradient error census at the BASELINE-sized goldens (GPU box).

For each golden: the oracle in float64 (exact yardstick), the oracle in fp32 (ATen fp32,
what the reference computes), the HIP path in fp32 and in bf16 AMP.  Prints, per
parameter, the relative L2 distance of each fp32/bf16 gradient from the float64 one, and
writes the table to gpurun_out/sized_diag_<name>.json.

    python scripts/sized_diag.py c2_b2 c3_b2 amp_hybrid
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "espnet-1_amd"), ROOT]

import torch  # noqa: E402

from goldens import is_null_grad, regenerate_sized, section  # noqa: E402
from test_model_build import build  # noqa: E402
from oracle.asr_oracle import OracleASR  # noqa: E402


def rel(a, b):
    a, b = a.double(), b.double()
    n = b.norm().item()
    return (a - b).norm().item() / n if n else (a - b).norm().item()


def main():
    torch.set_num_threads(16)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    for name in sys.argv[1:]:
        cfg, d, m = regenerate_sized(name, build)
        state = {k: v.detach().clone() for k, v in m.state_dict().items()}
        inp = {k: torch.from_numpy(v) for k, v in section(d, "in").items()}
        res = {}
        for tag, dt in (("o64", torch.float64), ("o32", torch.float32)):
            ora = OracleASR(cfg, state, dtype=dt)
            loss, _, _ = ora(**{k: v.clone() for k, v in inp.items()})
            loss.backward()
            res[tag] = (float(loss), {k: p.grad.detach().double() for k, p in ora.params.items()},
                        ora.encoder_out.detach().double())
        for tag, amp in (("hip32", False), ("hipamp", True)):
            _, _, mm = regenerate_sized(name, build)
            mm.prepare("cuda:0", amp=amp)
            mm.train()
            loss, _, _ = mm(**{k: v.clone() for k, v in inp.items()})
            loss.backward()
            torch.cuda.synchronize()
            res[tag] = (float(loss), {k: p.grad.detach().cpu().double() for k, p in mm.named_parameters()},
                        mm._last_encoder_out[0].detach().cpu().double())
            del mm
            torch.cuda.empty_cache()
        ampdev = section(d, "ampdev")
        l64, g64, e64 = res["o64"]
        rows = []
        for k in g64:
            if is_null_grad(k):
                continue
            rows.append(dict(k=k, o32=rel(res["o32"][1][k], g64[k]), hip32=rel(res["hip32"][1][k], g64[k]),
                             hipamp=rel(res["hipamp"][1][k], g64[k]), refamp=float(ampdev[k])))
        summary = {t: dict(loss=res[t][0], loss_rel=abs(res[t][0] - l64) / abs(l64),
                           enc_maxabs=float((res[t][2] - e64).abs().max())) for t in ("o32", "hip32", "hipamp")}
        summary["ref_amp_loss_rel"] = abs(float(d["amp.loss"]) - float(d["out.loss"])) / abs(float(d["out.loss"]))
        with open(os.path.join(ROOT, "gpurun_out", f"sized_diag_{name}.json"), "w") as f:
            json.dump(dict(summary=summary, rows=rows), f)
        print(name, json.dumps(summary))
        for key in ("o32", "hip32", "hipamp"):
            v = sorted(r[key] for r in rows)
            print(f"  {key:7s} relL2 vs f64: median {v[len(v) // 2]:.2e} p90 {v[int(len(v) * .9)]:.2e} max {v[-1]:.2e}")
        rr = sorted(rows, key=lambda r: -r["hip32"] / max(r["o32"], 1e-12))
        print("  worst hip32/o32:", "; ".join(f"{r['k']} {r['hip32']:.1e}/{r['o32']:.1e}" for r in rr[:6]))
        ra = sorted(rows, key=lambda r: -r["hipamp"] / max(r["refamp"], 1e-12))
        print("  worst hipamp/refamp:", "; ".join(f"{r['k']} {r['hipamp']:.1e}/{r['refamp']:.1e}" for r in ra[:6]))


if __name__ == "__main__":
    main()

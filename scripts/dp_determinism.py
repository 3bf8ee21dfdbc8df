"""Run-to-run determinism of the 2-rank gloo DP training loop on one GPU (the ragged-shard
test's workers, tests/test_dp_ragged_gpu.py): N runs of one mode, every run's final arena
compared with the first run's.  usage: dp_determinism.py MODE N"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402

import test_dp_ragged_gpu as T  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "eager"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    env = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("EA_"))
    ref = T._run(mode)
    bad = 0
    for i in range(1, n):
        r = T._run(mode)
        for k in (0, 1):
            if not torch.equal(r[k]["w"], ref[k]["w"]):
                bad += 1
                print(f"[{env}] {mode} run {i} rank {k}: {T._wdiff(r[k], ref[k])[:300]}", flush=True)
    print(f"[{env}] {mode}: {bad} mismatching rank-runs of {2 * (n - 1)}", flush=True)


if __name__ == "__main__":
    main()

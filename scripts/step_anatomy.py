"""Step anatomy from a rocprofv3 kernel trace (CSV): one step between two Adam launches,
per-queue busy time, idle gaps, and the main queue's time by kernel family."""
import collections
import csv
import re
import sys


def family(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"^void ", "", n)
    m = re.match(r"([A-Za-z0-9_]+)(<[^(]*>)?", n)
    base = m.group(1) if m else n[:40]
    if base.startswith("_ZN"):
        mm = re.search(r"N_1\d*([a-z_0-9]+?)(I|E)", n)
        base = mm.group(1) if mm else base[:40]
    tmpl = (m.group(2) or "")[:40] if m else ""
    return base + tmpl


def main(path, which=-2):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    a, b = adam[which - 1], adam[which]
    step = rows[a + 1: b + 1]
    t0 = int(rows[a]["End_Timestamp"])
    t1 = int(step[-1]["End_Timestamp"])
    print(f"step wall {(t1 - t0) / 1e3:.1f} us, {len(step)} kernels")
    byq = collections.defaultdict(list)
    for r in step:
        byq[r["Queue_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    # union busy
    iv = sorted((s, e) for q in byq.values() for s, e, _ in q)
    busy, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    print(f"some queue busy {busy / 1e3:.1f} us; idle {(t1 - t0 - busy) / 1e3:.1f} us")
    for q, ks in sorted(byq.items()):
        tot = sum(e - s for s, e, _ in ks)
        fam = collections.Counter()
        cnt = collections.Counter()
        for s, e, n in ks:
            fam[family(n)] += e - s
            cnt[family(n)] += 1
        print(f"queue {q}: {len(ks)} kernels, {tot / 1e3:.1f} us")
        for f, t in fam.most_common(25):
            print(f"   {t / 1e3:8.1f} us  x{cnt[f]:4d}  {f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else -2)

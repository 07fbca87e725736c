"""Timeline of the comm-bound ViT-H DP iteration from a rocprofv3 kernel trace.

usage: python scripts/probes/vit_timeline.py <kernel_trace.csv> [table_fwd_us table_bwd_bucket_us]

Splits the trace into iterations at the forward deadline GEMM (the one
compute kernel longer than 0.6x the table forward time),
then prints, for the last 3 iterations, every kernel with its start
offset, duration and the idle gap in front of it, and a summary: iteration
span, sum of deadline-kernel time, time between iterations (host sync +
relaunch), and per-kernel overshoot over the table durations."""
import csv
import sys
from collections import defaultdict


def short(n: str) -> str:
    n = n.replace("(anonymous namespace)::", "").split("(")[0]
    return n[-60:]


def main() -> None:
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                  r.get("Queue_Id", r.get("Stream_Id", "?"))) for r in rows), key=lambda k: k[0])
    fwd_us = float(sys.argv[2]) if len(sys.argv) > 2 else None
    bwd_us = float(sys.argv[3]) if len(sys.argv) > 3 else None
    # iteration starts: the forward GEMM (the one compute kernel longer than
    # 0.6x the forward time; the backward buckets are 4x shorter)
    lim = 0.6 * (fwd_us or 2000.0) * 1e3
    starts = [i for i, (s, e, n, q) in enumerate(ks) if "gemm" in n and e - s > lim]
    print(f"{len(ks)} kernels, {len(starts)} iteration starts")
    hist = defaultdict(lambda: [0, 0.0])
    for s, e, n, q in ks:
        hist[(n, q)][0] += 1
        hist[(n, q)][1] += (e - s) / 1e3
    for (n, q), (c, t) in sorted(hist.items(), key=lambda kv: -kv[1][1]):
        print(f"  q{q:>3} {c:6d} calls {t / 1e3:9.3f} ms  {n}")
    if len(starts) < 4:
        starts = [0]
    iters = []
    for j in range(len(starts)):
        lo = starts[j]
        hi = starts[j + 1] if j + 1 < len(starts) else len(ks)
        iters.append(ks[lo:hi])
    for it in iters[-4:-1]:
        t0 = it[0][0]
        print("---- iteration")
        prev_end = defaultdict(lambda: t0)
        for s, e, n, q in it:
            print(f"  q{q:>3} +{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:9.1f}  gap {(s - prev_end[q]) / 1e3:7.1f}  {n}")
            prev_end[q] = e
    # summary over all full iterations but the first 5
    spans, between, dl = [], [], []
    for j in range(5, len(iters) - 1):
        it, nxt = iters[j], iters[j + 1]
        end = max(e for _, e, _, _ in it)
        spans.append((end - it[0][0]) / 1e3)
        between.append((nxt[0][0] - end) / 1e3)
        dl.append([(e - s) / 1e3 for s, e, n, _ in it if "gemm" in n])
    if spans:
        m = len(spans)
        print(f"iterations {m}: span {sum(spans) / m:.1f} us, gap to next {sum(between) / m:.1f} us, "
              f"period {(sum(spans) + sum(between)) / m:.1f} us")
        per = [sum(x) / m for x in zip(*dl)] if all(len(d) == len(dl[0]) for d in dl) else []
        if per:
            print("deadline kernel durations (mean): " + ", ".join(f"{x:.1f}" for x in per))
            if fwd_us and bwd_us:
                tgt = [fwd_us] + [bwd_us] * (len(per) - 1)
                print("overshoot vs table (us): " + ", ".join(f"{a - b:+.1f}" for a, b in zip(per, tgt)))


if __name__ == "__main__":
    main()

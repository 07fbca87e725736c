#!/usr/bin/env python3
"""xgmi kernels vs the local HBM copy roofline, from scripts/xgmi_sweep.sh output.

Ranks share one GPU, so every byte a kernel moves is local HBM traffic. Per
rank and operation the kernels' traffic is fixed by their data path
(csrc/kernels/xgmi.hip; n = bytes per rank block, W ranks):
  all_gather      push n to W-1 peers + own recv, copy W-1 slots out  n(3W-1)
  reduce_scatter  push W-1 blocks, reduce W sources into recv         n(3W-1)
  all_to_all      push W-1 blocks, own block, copy W-1 slots out      n(4W-2)
  all_reduce      two-shot: scatter, reduce + broadcast, copy out     n(6W-4)/W  (n = whole message)
  sendrecv        ring: push n into the next rank's window, copy n out of mine   4n
  copy            hipMemcpyAsync D2D                                  2n
With registered buffers (EXTRA=--registered: zero-copy paths) the same ops move
  all_gather      one load, W stores straight into every rank's receive buffer  n(W+1)
  reduce_scatter  W loads straight out of every rank's send buffer, one store   n(W+1)
  all_reduce      chunk r of W send buffers summed into W receive buffers       2n
  all_to_all      (staged, as above)                                            n(4W-2)
All W ranks run the op at the same time, so the GPU moves W x that; the copy
line of the same sweep (all ranks copying at once) is the roofline.

    python scripts/xgmi_roofline.py gpurun_out/xgmi_sweep.jsonl [--blocks 256]
"""
import argparse
import collections
import json


def traffic(op, n, W, registered=False):
    if registered and op in ("all_gather", "reduce_scatter"):
        return n * (W + 1)
    if registered and op == "all_reduce" and n > 256 * 1024 and n % 16 == 0:
        return 2 * n
    return {"all_gather": n * (3 * W - 1), "reduce_scatter": n * (3 * W - 1), "all_to_all": n * (4 * W - 2),
            "all_reduce": n * (6 * W - 4) / W, "sendrecv": 4 * n, "copy": 2 * n}[op]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("jsonl")
    ap.add_argument("--blocks", type=int, default=None, help="only this block cap (default: best per op)")
    a = ap.parse_args()
    rows = [json.loads(l) for l in open(a.jsonl) if l.strip()]
    best = collections.OrderedDict()
    for r in rows:
        if r.get("commtest") != "bench" or (a.blocks and r.get("blocks") != a.blocks):
            continue
        W, op, count = r["W"], r["op"], r["count"]
        es = r["bytes"] / count / (1 if op in ("all_reduce", "copy", "sendrecv") else W)
        n = count * es
        t = r["time_us"] * 1e-6
        reg = "--registered" in (r.get("extra") or "")
        hbm = W * traffic(op, n, W, reg) / t / 1e9  # whole-GPU GB/s
        key = (W, count, op, reg)
        if key not in best or hbm > best[key]["hbm"]:
            best[key] = {"hbm": hbm, "algbw": r["algbw_GBps"], "t": r["time_us"], "blocks": r.get("blocks"),
                         "mem": r.get("mem")}
    print("| W | elements/rank | op | buffers | blocks | time (us) | algbw GB/s | GPU HBM GB/s (model) | % of copy |")
    print("|---:|---:|---|---|---:|---:|---:|---:|---:|")
    for (W, count, op, reg), v in sorted(best.items(), key=lambda kv: kv[0]):
        roof = best.get((W, count, "copy", reg), {}).get("hbm")
        pct = f"{100 * v['hbm'] / roof:.0f} %" if roof and op != "copy" else "—"
        print(f"| {W} | {count} | {op} | {'registered' if reg else 'staged'} | {v['blocks']} | {v['t']:.1f} | "
              f"{v['algbw']:.0f} | {v['hbm']:.0f} | {pct} |")


if __name__ == "__main__":
    main()

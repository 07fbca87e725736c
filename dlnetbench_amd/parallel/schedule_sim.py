"""Discrete-event model of the pipeline schedules' enqueue logic.

Mirrors csrc/src/strategy_pipeline.cpp (enqueue_gpipe / enqueue_1f1b /
enqueue_interleaved / enqueue_dualpipe): per rank a compute stream and two link streams (prev,
next) executing their operations in order; compute waits on receive events
and on the send of the buffer it overwrites; a link operation is a group of
at most one send and one receive that completes when every matching
operation (per channel FIFO order) sits at the head of its own stream with
its waits satisfied. By default links cost nothing, so a finished run's
makespan is the schedule's compute critical path and a stuck run is a
deadlock; with `link` > 0 every link group takes that long (the xGMI cost
model's send/recv time: xgmi_model.predict_hybrid).

    python -m dlnetbench_amd.parallel.schedule_sim --stages 4 --microbatches 8 --virtual 2
"""
from __future__ import annotations

import argparse
from typing import Dict, List, Tuple


def build(S: int, mb: int, V: int, f: float, b: float, sched: str,
          link: float = 0.0) -> Dict[Tuple[int, str], List[dict]]:
    streams: Dict[Tuple[int, str], List[dict]] = {}
    total = mb * V

    def op(r, st, **kw):
        streams.setdefault((r, st), []).append(kw)

    for s in range(S):
        il = sched == "interleaved"

        def chunk_f(k):
            return (k // S) % V

        def chunk_b(k):
            return V - 1 - (k // S) % V

        def in_f(k):
            return not (s == 0 and chunk_f(k) == 0) if il else s > 0

        def out_f(k):
            return not (s == S - 1 and chunk_f(k) == V - 1) if il else s < S - 1

        def in_b(k):
            return not (s == S - 1 and chunk_b(k) == V - 1) if il else s < S - 1

        def out_b(k):
            return not (s == 0 and chunk_b(k) == 0) if il else s > 0

        def fwd(k):
            waits = [(s, "recvF", k)] if S > 1 and in_f(k) else []
            if k >= 2 and S > 1 and out_f(k - 2):
                waits.append((s, "sentF", k - 2))
            op(s, "c", dur=f / V, waits=waits, rec=[(s, "fdone", k)])

        def bwd(j):
            waits = [(s, "recvB", j)] if S > 1 and in_b(j) else []
            if j >= 2 and S > 1 and out_b(j - 2):
                waits.append((s, "sentB", j - 2))
            op(s, "c", dur=b / V, waits=waits, rec=[(s, "bdone", j)])

        def nxt(sf, rb):  # next link: send F(sf) to s+1, receive B(rb) from s+1
            if S == 1 or (sf < 0 and rb < 0):
                return
            waits, p2p, rec = [], [], []
            if sf >= 0:
                waits.append((s, "fdone", sf)); p2p.append(("send", "F", (s + 1) % S)); rec.append((s, "sentF", sf))
            if rb >= 0:
                if rb >= 2:
                    waits.append((s, "bdone", rb - 2))
                p2p.append(("recv", "B", (s + 1) % S)); rec.append((s, "recvB", rb))
            op(s, "n", dur=link, waits=waits, rec=rec, p2p=p2p)

        def prv(sb, rf):  # previous link: send B(sb) to s-1, receive F(rf) from s-1
            if S == 1 or (sb < 0 and rf < 0):
                return
            waits, p2p, rec = [], [], []
            if sb >= 0:
                waits.append((s, "bdone", sb)); p2p.append(("send", "B", (s - 1) % S)); rec.append((s, "sentB", sb))
            if rf >= 0:
                if rf >= 2:
                    waits.append((s, "fdone", rf - 2))
                p2p.append(("recv", "F", (s - 1) % S)); rec.append((s, "recvF", rf))
            op(s, "p", dur=link, waits=waits, rec=rec, p2p=p2p)

        if il:
            w = total if mb == S else min((S - s - 1) * 2 + (V - 1) * S, total)
            rem = total - w
            if in_f(0):
                prv(-1, 0)
            for k in range(w):
                fwd(k)
                nxt(k if out_f(k) else -1, 0 if (k == w - 1 and rem > 0 and in_b(0)) else -1)
                prv(-1, k + 1 if k + 1 < total and in_f(k + 1) else -1)
            for j in range(rem):
                k = w + j
                fwd(k)
                bwd(j)
                nxt(k if out_f(k) else -1, j + 1 if j + 1 < total and in_b(j + 1) else -1)
                prv(j if out_b(j) else -1, k + 1 if k + 1 < total and in_f(k + 1) else -1)
            if rem == 0 and in_b(0):
                nxt(-1, 0)
            for j in range(rem, total):
                bwd(j)
                nxt(-1, j + 1 if j + 1 < total and in_b(j + 1) else -1)
                prv(j if out_b(j) else -1, -1)
        elif sched == "1f1b":
            w = min(S - s - 1, mb)
            steady = mb - w
            for i in range(w):
                prv(-1, i) if s > 0 else None
                fwd(i)
                nxt(i, -1) if s < S - 1 else None
            if steady > 0 and s > 0:
                prv(-1, w)
            for j in range(steady):
                i = w + j
                fwd(i)
                nxt(i, j) if s < S - 1 else None
                bwd(j)
                prv(j, i + 1 if j + 1 < steady else -1) if s > 0 else None
            for j in range(steady, mb):
                nxt(-1, j) if s < S - 1 else None
                bwd(j)
                prv(j, -1) if s > 0 else None
        else:  # gpipe
            for i in range(mb):
                prv(-1, i) if s > 0 else None
                fwd(i)
                nxt(i, -1) if s < S - 1 else None
            for j in range(mb):
                nxt(-1, j) if s < S - 1 else None
                bwd(j)
                prv(j, -1) if s > 0 else None
    return streams


def dualpipe_ticks(S: int, mb: int) -> List[List[tuple]]:
    """The DualPipe tick schedule (build_dualpipe in strategy_pipeline.cpp): row t holds, per stage, None or
    (dir, microbatch, is_backward). dir 0 = the "down" copy (stage s at position s), 1 = the "up" copy
    (position S-1-s); mb/2 microbatches per copy. A forward within the 1F1B in-flight cap S - position
    (the copy with fewer forwards issued first), else the oldest ready backward."""
    H = mb // 2

    def pos(s, d):
        return s if d == 0 else S - 1 - s

    fdone, bdone = {}, {}
    nf = [[0, 0] for _ in range(S)]
    nb = [[0, 0] for _ in range(S)]
    ticks, remaining, t = [], S * 2 * H * 2, 0
    while remaining:
        assert t < 16 * (mb + S) + 64, "dualpipe schedule did not converge"
        row = []
        for s in range(S):
            best = None
            order = [0, 1]
            if nf[s][1] < nf[s][0] or (nf[s][1] == nf[s][0] and pos(s, 1) < pos(s, 0)):
                order = [1, 0]
            for d in order:
                i = nf[s][d]
                if i >= H or i - nb[s][d] >= S - pos(s, d):
                    continue
                if pos(s, d) > 0 and fdone.get((s - 1 if d == 0 else s + 1, d, i), t) >= t:
                    continue
                best = (d, i, False)
                break
            if best is None:
                for d in (0, 1):
                    i = nb[s][d]
                    if i >= nf[s][d] or fdone.get((s, d, i), t) >= t:
                        continue
                    if pos(s, d) < S - 1 and bdone.get((s + 1 if d == 0 else s - 1, d, i), t) >= t:
                        continue
                    if best is None or i < best[1]:
                        best = (d, i, True)
            if best is not None:
                d, i, bw = best
                if bw:
                    bdone[(s, d, i)] = t
                    nb[s][d] += 1
                else:
                    fdone[(s, d, i)] = t
                    nf[s][d] += 1
                remaining -= 1
            row.append(best)
        ticks.append(row)
        t += 1
    return ticks


def dualpipe_floor(S: int, mb: int, f: float, b: float) -> float:
    """Compute-only makespan of the tick order (the driver's compute_floor_us for dualpipe)."""
    ffin, bfin, free, span = {}, {}, [0.0] * S, 0.0
    for row in dualpipe_ticks(S, mb):
        for s, op in enumerate(row):
            if op is None:
                continue
            d, i, bw = op
            start = free[s]
            up, down = (s - 1, s + 1) if d == 0 else (s + 1, s - 1)
            pos = s if d == 0 else S - 1 - s
            if not bw:
                if pos > 0:
                    start = max(start, ffin[(up, d, i)])
                ffin[(s, d, i)] = free[s] = start + f
            else:
                start = max(start, ffin[(s, d, i)])
                if pos < S - 1:
                    start = max(start, bfin[(down, d, i)])
                bfin[(s, d, i)] = free[s] = start + b
            span = max(span, free[s])
    return span


def build_dualpipe(S: int, mb: int, f: float, b: float, link: float = 0.0) -> Dict[Tuple[int, str], List[dict]]:
    """Streams of enqueue_dualpipe: per tick the rank's op on the compute stream (waiting on its input's
    receive), then the next-link group, then the previous-link group - each at most one send (this rank's
    op output) and one receive (the neighbour's op output of the same tick, into a buffer of its own).
    One FIFO channel per link direction, as one communicator per link carries every message type."""
    streams: Dict[Tuple[int, str], List[dict]] = {}
    H = mb // 2

    def pos(s, d):
        return s if d == 0 else S - 1 - s

    def travels(s, op, towards_next):  # does op's output at stage s go over that link?
        if op is None:
            return False
        d, _, bw = op
        if ((d == 0) != bw) != towards_next:
            return False
        return pos(s, d) > 0 if bw else pos(s, d) < S - 1

    for row in dualpipe_ticks(S, mb):
        for s in range(S):
            op = row[s]
            if op is not None:
                d, i, bw = op
                k = d * H + i
                needs = (pos(s, d) < S - 1) if bw else (pos(s, d) > 0)
                waits = [(s, "recvB" if bw else "recvF", k)] if needs else []
                streams.setdefault((s, "c"), []).append(
                    {"dur": b if bw else f, "waits": waits, "rec": [(s, "bdone" if bw else "fdone", k)]})
            for nxt, st in ((True, "n"), (False, "p")):
                peer = s + 1 if nxt else s - 1
                if not 0 <= peer < S:
                    continue
                theirs = row[peer]
                send, recv = travels(s, op, nxt), travels(peer, theirs, not nxt)
                if not (send or recv):
                    continue
                waits, p2p, rec = [], [], []
                if send:
                    d, i, bw = op
                    waits.append((s, "bdone" if bw else "fdone", d * H + i))
                    p2p.append(("send", "L", peer))
                    rec.append((s, "sent", (d, i, bw)))
                if recv:
                    d, i, bw = theirs
                    p2p.append(("recv", "L", peer))
                    rec.append((s, "recvB" if bw else "recvF", d * H + i))
                streams.setdefault((s, st), []).append({"dur": link, "waits": waits, "rec": rec, "p2p": p2p})
    return streams


def simulate(streams, semantics: str = "rendezvous") -> Tuple[float, List[Tuple[int, str]]]:
    """Returns (makespan, streams left unfinished = deadlock).

    semantics: "rendezvous" (NCCL/RCCL-like and the strictest: a group completes only when every matching
    operation's group sits at the head of its stream) or "buffered" (the xgmi / shared-memory backends:
    a send needs only the receiver to have consumed message seq-2 of its channel, a receive needs the
    matching send done, and a group's operations run one after the other in issue order)."""
    if semantics == "buffered":
        return _simulate_buffered(streams)
    posted: Dict[tuple, int] = {}
    for key, ops in streams.items():
        for o in ops:
            for kind, d, peer in o.get("p2p", []):
                ch = (key[0], peer, d) if kind == "send" else (peer, key[0], d)
                n = posted.get((ch, kind), 0)
                o.setdefault("tags", []).append((ch, kind, n))
                posted[(ch, kind)] = n + 1
    done: Dict[tuple, float] = {}
    heads = {k: 0 for k in streams}
    free = {k: 0.0 for k in streams}
    t_end, progress = 0.0, True
    while progress:
        progress = False
        ready = {}
        for key, ops in streams.items():
            if heads[key] < len(ops):
                o = ops[heads[key]]
                if all(w in done for w in o["waits"]):
                    ready[key] = max([free[key]] + [done[w] for w in o["waits"]])
        for key in ready:
            group, todo, ok = {key}, [key], True
            while todo and ok:
                k1 = todo.pop()
                for ch, kind, n in streams[k1][heads[k1]].get("tags", []):
                    other = "recv" if kind == "send" else "send"
                    hit = [k2 for k2 in ready if (ch, other, n) in streams[k2][heads[k2]].get("tags", [])]
                    if not hit:
                        ok = False
                        break
                    for k2 in hit:
                        if k2 not in group:
                            group.add(k2)
                            todo.append(k2)
            if not ok:
                continue
            t = max(ready[k] for k in group)
            for k in group:
                o = streams[k][heads[k]]
                fin = t + o["dur"]
                for e in o["rec"]:
                    done[e] = fin
                free[k] = fin
                heads[k] += 1
                t_end = max(t_end, fin)
            progress = True
            break
    return t_end, [k for k in streams if heads[k] < len(streams[k])]


def _simulate_buffered(streams, slots: int = 2) -> Tuple[float, List[Tuple[int, str]]]:
    seq = {}
    for key, ops in streams.items():
        lst = []
        for o in ops:  # a group becomes its operations, in issue order (sends first, as the backends do)
            p2p = o.get("p2p")
            if not p2p:
                lst.append(o)
                continue
            order = sorted(range(len(p2p)), key=lambda i: p2p[i][0] != "send")
            for n, i in enumerate(order):
                kind, d, peer = p2p[i]
                ch = (key[0], peer, d) if kind == "send" else (peer, key[0], d)
                m = seq.get((ch, kind), 0)
                seq[(ch, kind)] = m + 1
                lst.append({"dur": 0.0, "waits": o["waits"] if n == 0 else [], "rec": [o["rec"][i]],
                            "msg": (ch, kind, m)})
        streams_key = key
        seq_streams = lst
        streams = dict(streams)
        streams[streams_key] = seq_streams
    sent: Dict[tuple, float] = {}
    consumed: Dict[tuple, float] = {}
    done: Dict[tuple, float] = {}
    heads = {k: 0 for k in streams}
    free = {k: 0.0 for k in streams}
    t_end, progress = 0.0, True
    while progress:
        progress = False
        for key, ops in streams.items():
            while heads[key] < len(ops):
                o = ops[heads[key]]
                if not all(w in done for w in o["waits"]):
                    break
                t = max([free[key]] + [done[w] for w in o["waits"]])
                if "msg" in o:
                    ch, kind, m = o["msg"]
                    if kind == "send":
                        if m >= slots and (ch, m - slots) not in consumed:
                            break
                        t = max(t, consumed.get((ch, m - slots), 0.0))
                        sent[(ch, m)] = t
                    else:
                        if (ch, m) not in sent:
                            break
                        t = max(t, sent[(ch, m)])
                        consumed[(ch, m)] = t
                fin = t + o["dur"]
                for e in o["rec"]:
                    done[e] = fin
                free[key] = fin
                heads[key] += 1
                t_end = max(t_end, fin)
                progress = True
    return t_end, [k for k in streams if heads[k] < len(streams[k])]


def floor(S: int, mb: int, V: int, f: float, b: float) -> float:
    """The driver's compute floor (compute_floor_us): (mb + (S-1)/V)(f_mb + b_mb), f/b per microbatch."""
    return (mb + (S - 1) / V) * (f + b)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--stages", type=int, default=4)
    ap.add_argument("--microbatches", type=int, default=8)
    ap.add_argument("--virtual", type=int, default=2)
    ap.add_argument("--fwd", type=float, default=1.0, help="forward time of one microbatch on one stage")
    ap.add_argument("--bwd", type=float, default=2.0)
    a = ap.parse_args(argv)
    for sched, V in (("gpipe", 1), ("1f1b", 1), ("interleaved", a.virtual)):
        t, stuck = simulate(build(a.stages, a.microbatches, V, a.fwd, a.bwd, sched))
        print(f"{sched:12s} V={V}: makespan {t:.3f}  floor {floor(a.stages, a.microbatches, V, a.fwd, a.bwd):.3f}"
              + (f"  DEADLOCK {stuck[:4]}" if stuck else ""))
    if a.stages % 2 == 0 and a.microbatches % 2 == 0:
        t, stuck = simulate(build_dualpipe(a.stages, a.microbatches, a.fwd, a.bwd))
        print(f"{'dualpipe':12s} V=1: makespan {t:.3f}  floor "
              f"{dualpipe_floor(a.stages, a.microbatches, a.fwd, a.bwd):.3f}" + (f"  DEADLOCK {stuck[:4]}" if stuck else ""))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

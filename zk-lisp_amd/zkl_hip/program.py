"""`zk-lisp prove`'s segment loop on one device (prove.rs:1000-1175): every segment of a program
built on host threads by the per-segment builder (zkl_build_segment_trace, no full trace) straight
into a context's pinned trace buffer (zkl_hip_trace_buffer), proved through the host-trace entry
point (zkl_hip_prove_segment: the columns DMA'd from that buffer, overlapped with their LDE) by
`inflight` contexts -- the reference's bounded rayon pool (prove.rs:1018-1050) -- and wrapped as
zl1 step proofs.

Per context the next segment is built into the second buffer slot while the current one proves,
so host building (~0.2 s per 65,536-row segment on one thread) overlaps the GPU.
"""
from __future__ import annotations

import threading
import time
from concurrent.futures import ThreadPoolExecutor

from . import Context, Program, proof_options, step_info_for, step_proof_encode


class SegmentProof:
    __slots__ = ("index", "rows", "width", "pi", "state_in", "state_out", "opts", "proof", "build_ms", "prove_ms")

    def __init__(self, index, rows, width, pi, state_in, state_out, opts):
        self.index, self.rows, self.width, self.pi = index, rows, width, pi
        self.state_in, self.state_out, self.opts = state_in, state_out, opts
        self.proof = None
        self.build_ms = self.prove_ms = 0.0


def prove_program(program: Program, plan, device: int = 0, inflight: int = 4, builders: int = 8, segments=None,
                  queries: int = 64, blowup: int = 16, grind: int = 16, contexts=None, on_proof=None):
    """Proves the segments of `plan` ([(r_start, r_end)], zkl_plan_segments) whose indices are in
    `segments` (default all): returns {index: SegmentProof}.  `contexts` may pass existing
    Contexts (then `inflight` = their count and they stay open).  on_proof(SegmentProof) runs in
    the proving thread after each proof."""
    idx = list(range(len(plan))) if segments is None else list(segments)
    own = contexts is None
    ctxs = [Context(device) for _ in range(inflight)] if own else list(contexts)
    inflight = len(ctxs)
    # both buffer slots of every context sized once for the widest, longest segment (the full
    # trace's width bounds every segment layout): the builders then never wait on a context
    # that is proving
    cap = program.width * max(b - a for a, b in plan) * 16
    bufs = [[c.trace_buffer(cap, slot) for slot in (0, 1)] for c in ctxs]
    pool = ThreadPoolExecutor(max_workers=max(1, builders))
    out, errors = {}, []
    lock = threading.Lock()

    def build(k, slot, i):
        a, b = plan[i]
        m = b - a
        t0 = time.perf_counter()
        buf = bufs[k][slot]
        pi, w, sin, sout = program.segment_into(a, b, buf)
        rec = SegmentProof(i, (a, b), w, pi, sin, sout, proof_options(w, m, queries=queries, blowup=blowup,
                                                                           grind=grind))
        rec.build_ms = (time.perf_counter() - t0) * 1e3
        return rec, buf

    def work(k):
        ctx = ctxs[k]
        mine = idx[k::inflight]
        try:
            nxt = pool.submit(build, k, 0, mine[0]) if mine else None
            for j in range(len(mine)):
                rec, buf = nxt.result()
                nxt = pool.submit(build, k, (j + 1) % 2, mine[j + 1]) if j + 1 < len(mine) else None
                t0 = time.perf_counter()
                rec.proof = ctx.prove_segment(buf, rec.width, rec.rows[1] - rec.rows[0], rec.pi, rec.opts)
                rec.prove_ms = (time.perf_counter() - t0) * 1e3
                if on_proof is not None:
                    on_proof(rec)
                with lock:
                    out[rec.index] = rec
        except Exception as e:  # noqa: BLE001  (re-raised below, after every worker stopped)
            with lock:
                errors.append(e)
            if nxt is not None:
                try:
                    nxt.result()
                except Exception:  # noqa: BLE001
                    pass

    th = [threading.Thread(target=work, args=(k,)) for k in range(inflight)]
    try:
        for x in th:
            x.start()
        for x in th:
            x.join()
    finally:
        pool.shutdown(wait=True)
        if own:
            for c in ctxs:
                c.close()
    if errors:
        raise errors[0]
    return out


def steps_of(records, total: int, main_args=()):
    """The zl1 step proofs (ZKLSTP1) of proved segments, in index order (prove.rs:1144-1174)."""
    return [step_proof_encode(r.pi, step_info_for(r.pi, r.index, total, r.state_in, r.state_out, main_args=main_args),
                              r.proof) for r in sorted(records, key=lambda r: r.index)]

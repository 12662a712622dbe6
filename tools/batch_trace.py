"""Summarise an SHD_BATCH_TRACE file (sssp_batch_kernel: per batch {start, end} ticks of
wall_clock64 (100 MHz), slot, near iterations, sweeps, expansions, relaxations, sources; then per
batch position {source, pi}): span of each launch, batch durations, the idle tail of the slots
(time between a slot's last batch end and the kernel's last batch end), and how the batch
duration correlates with the batch's counters and its sources' pi.

usage: python tools/batch_trace.py FILE
"""
import sys

import numpy as np

TICK_MS = 1e-5  # wall_clock64 (s_memrealtime) counts at 100 MHz

raw = np.fromfile(sys.argv[1], dtype=np.int64)
i = 0
launch = 0
while i < len(raw):
    nb, kf, slots, rows = (int(x) for x in raw[i:i + 4])
    W = 12  # kBTraceWords
    bt = raw[i + 4:i + 4 + W * nb].reshape(nb, W).astype(np.float64)
    i += 4 + W * nb
    sp = raw[i:i + 2 * rows].reshape(rows, 2)
    i += 2 * rows
    src = sp[:, 0]
    pi = sp[:, 1].copy().view(np.float64)
    st, en, sl = bt[:, 0], bt[:, 1], bt[:, 2].astype(int)
    t0, t1 = st.min(), en.max()
    span = (t1 - t0) * TICK_MS
    dur = (en - st) * TICK_MS
    ph = np.stack([bt[:, 8] - st, bt[:, 9] - bt[:, 8], bt[:, 10] - bt[:, 9], en - bt[:, 10]],
                  axis=1) * TICK_MS  # SSSP, parents, epilogue, reset
    used = np.unique(sl)
    last = np.array([en[sl == s].max() for s in used])
    first = np.array([st[sl == s].min() for s in used])
    idle_tail = (t1 - last) * TICK_MS
    idle_head = (first - t0) * TICK_MS
    busy = dur.sum()
    print("launch %d: %d batches of %d, %d slots used of %d, span %.2f ms" %
          (launch, nb, kf, len(used), slots, span))
    q = np.percentile(dur, [0, 10, 50, 90, 100])
    slow = np.argsort(dur)[-max(1, nb // 20):]
    print("  phases ms (SSSP, parents, epilogue, reset): mean %s; slowest 5 %% of batches %s" % (
        " ".join("%.2f" % x for x in ph.mean(axis=0)),
        " ".join("%.2f" % x for x in ph[slow].mean(axis=0))))
    print("  batch ms: min %.2f p10 %.2f median %.2f p90 %.2f max %.2f  mean %.2f" %
          (*q, dur.mean()))
    print("  busy %.1f %% of slots x span; idle tail mean %.2f ms max %.2f; idle head max %.2f ms" %
          (100 * busy / (len(used) * span), idle_tail.mean(), idle_tail.max(), idle_head.max()))
    # durations along the dequeue order (deciles)
    dec = np.array_split(dur, 10)
    print("  mean ms by dequeue decile:", " ".join("%.1f" % d.mean() for d in dec))
    order = np.argsort(st)
    k = max(1, nb // 20)
    print("  last %d batches dequeued: mean %.2f ms, ends %.2f..%.2f ms" %
          (k, dur[order[-k:]].mean(), (en[order[-k:]].min() - t0) * TICK_MS,
           (en[order[-k:]].max() - t0) * TICK_MS))
    feats = {"near it": bt[:, 3], "sweeps": bt[:, 4], "expansions": bt[:, 5],
             "relaxations": bt[:, 6], "sources": bt[:, 7]}
    pib = np.full((nb, int(bt[:, 7].max())), np.nan)
    off = np.concatenate([[0], np.cumsum(bt[:, 7].astype(int))])
    for b in range(nb):
        n = int(bt[b, 7])
        pib[b, :n] = pi[off[b]:off[b] + n]
    feats["pi mean"] = np.nanmean(pib, axis=1)
    feats["pi max"] = np.nanmax(pib, axis=1)
    feats["pi spread"] = np.nanmax(pib, axis=1) - np.nanmin(pib, axis=1)
    print("  corr(duration, x): " + ", ".join(
        "%s %.2f" % (k, np.corrcoef(dur, v)[0, 1]) for k, v in feats.items() if np.std(v) > 0))
    print("  per batch mean: " + ", ".join("%s %.4g" % (k, v.mean()) for k, v in feats.items()))
    np.savez(sys.argv[1] + ".%d.npz" % launch, dur=dur, start=st, end=en, slot=sl, src=src, pi=pi,
             cnt=bt[:, 3:8])
    launch += 1

#!/usr/bin/env python3
"""LDS bank-conflict model of k_scan_fast's table walk (CPU simulation).

Walks the builtin ruleset's k_scan_fast automaton the way the kernel does
(lane i of a 32-lane LDS group scans the i-th consecutive 4 KiB span of the
corpus, 7 bytes of warm-up) over text from the bench corpus generator, and
prices each step's ds_read_u16 under a row layout: a lane reads the dword at
row_dword[state] + col // 2, bank = dword % 32 (MI355X_MICROARCH.md §LDS,
ds_read_b32-class lane groups), cost = the most distinct dwords on one bank.

Usage: python tools/bank_sim.py [regions] [seed]
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import trivy_amd._native as N  # noqa: E402
import trivy_amd.secret as S  # noqa: E402

ROW = 134  # kFastRowBytes
SPAN = 4096


def image():
    sc = S.new_scanner(None)
    n = ctypes.c_size_t()
    oe = ctypes.c_uint32()
    N.check(N.lib.tsg_ruleset_scan_image(sc._rs.handle, None, 0, ctypes.byref(n), ctypes.byref(oe)))
    buf = (ctypes.c_uint8 * n.value)()
    N.check(N.lib.tsg_ruleset_scan_image(sc._rs.handle, buf, n.value, ctypes.byref(n), ctypes.byref(oe)))
    raw = np.frombuffer(bytes(buf), dtype=np.uint8)
    rows = len(raw) // ROW
    T = np.zeros((rows, 64), dtype=np.int32)
    for r in range(rows):
        T[r] = np.frombuffer(raw[r * ROW: r * ROW + 128].tobytes(), dtype=np.uint16)
    return T, oe.value


def fold6(b):
    return ((b << 1) & 0x3E) | (b & 0x40)


def corpus(regions, seed):
    size = regions * 32 * SPAN
    out = np.zeros(size, dtype=np.uint8)
    f, pos = 0, 0
    while pos < size:
        n = min(1 << 16, size - pos)
        buf = ctypes.create_string_buffer(n)
        N.check(N.gen.tsg_gen_file(seed, f, n, 1e-6, buf))
        out[pos: pos + n] = np.frombuffer(buf.raw, dtype=np.uint8)
        pos += n
        f += 1
    return out


def walk(T, text, regions):
    """states[lane, step], cols[lane, step] for lanes = regions * 32 spans."""
    lanes = regions * 32
    spans = text[: lanes * SPAN].reshape(lanes, SPAN)
    cols = fold6(spans.astype(np.int32)) >> 1
    st = np.zeros(lanes, dtype=np.int32)
    prev = np.zeros((lanes, 7), dtype=np.int32)
    prev[1:] = cols[:-1, -7:]
    for j in range(7):
        st = T[st, prev[:, j]]
    states = np.zeros((lanes, SPAN), dtype=np.int32)
    for j in range(SPAN):
        states[:, j] = st
        st = T[st, cols[:, j]]
    return states, cols


def cost(row_dword, states, cols):
    """Average LDS cycles per 32-lane group and step."""
    dw = row_dword[states] + (cols >> 1)  # lanes x steps
    lanes, steps = dw.shape
    g = dw.reshape(lanes // 32, 32, steps).transpose(0, 2, 1).reshape(-1, 32)
    g = np.sort(g, axis=1)
    distinct = np.ones_like(g, dtype=bool)
    distinct[:, 1:] = g[:, 1:] != g[:, :-1]
    bank = g % 32
    key = np.where(distinct, bank, 32)  # only distinct dwords count
    counts = np.zeros((g.shape[0], 33), dtype=np.int32)
    np.add.at(counts, (np.repeat(np.arange(g.shape[0]), 32), key.ravel()), 1)
    return counts[:, :32].max(axis=1).mean()


def main():
    regions = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 20261017
    T, oe = image()
    rows = T.shape[0]
    text = corpus(regions, seed)
    states, cols = walk(T, text, regions)
    hist = np.bincount(states.ravel(), minlength=rows) / states.size
    order = np.argsort(-hist)
    print(f"rows {rows}, out_entry {oe}, root share {hist[0]:.3f}, top16 {hist[order[:16]].sum():.3f}, "
          f"top32 {hist[order[:32]].sum():.3f}")
    cur = (np.arange(rows) * ROW) // 4
    print("stride 134 (current):", round(cost(cur, states, cols), 3))
    print("stride 128 (no rotation):", round(cost(np.arange(rows) * 32, states, cols), 3))
    rng = np.random.default_rng(1)
    print("random rotation:", round(cost(np.arange(rows) * 33 + rng.integers(0, 32, rows), states, cols), 3))


if __name__ == "__main__":
    main()


def optimize(states, cols, rows, hot=48, base_stride=33, rounds=2, seed=1):
    """Coordinate descent over the dword rotation of the `hot` most-visited
    rows (others keep base_stride packing): returns row_dword, cost."""
    hist = np.bincount(states.ravel(), minlength=rows)
    order = [int(s) for s in np.argsort(-hist)[:hot]]
    rot = {s: 0 for s in order}

    def layout():
        d = np.arange(rows) * base_stride
        for k, s in enumerate(order):  # hot rows: own 64-dword slots after the packed rows
            d[s] = rows * base_stride + 64 * k + rot[s]
        return d

    best = cost(layout(), states, cols)
    for _ in range(rounds):
        for s in order:
            cands = []
            for r in range(32):
                rot[s] = r
                cands.append((cost(layout(), states, cols), r))
            best, rot[s] = min(cands)
    return layout(), best


if __name__ == "__main__" and os.environ.get("BANK_OPT"):
    regions = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    T, oe = image()
    text = corpus(regions, 777)
    states, cols = walk(T, text, regions)
    text2 = corpus(regions, 31337)
    st2, co2 = walk(T, text2, regions)
    rows = T.shape[0]
    for stride in (33, 34):
        print("stride", stride * 4, "B:", round(cost(np.arange(rows) * stride, st2, co2), 3))
    d, c = optimize(states, cols, rows, hot=int(os.environ.get("BANK_HOT", "32")))
    print("optimized (train):", round(c, 3), " held-out:", round(cost(d, st2, co2), 3))

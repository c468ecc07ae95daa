"""Byte-range split of ONE large file, measured on one MI355X.

One synthetic file of --gb GB (bench.py's §8(d) text model, builtin secrets
planted at 1e-6/byte) is generated in HBM.  Timed, each with a device sync:
  whole   tsg_scan_device on the file (the single-GPU path);
  part r  tsg_scan_part_device over range r of W (the view is a pointer into
          the same buffer, as on a rank that received only its range);
  merge   tsg_scan_merge_device of the W parts on the owner.
With W GPUs the parts run concurrently, so the split step is projected as
max(part) + merge (+ the part blobs' transfer: KiB); the merge's findings are
checked equal to the whole-file scan's.  Prints one JSON line.

  python tools/split_bench.py --gb 5 --parts 2 4 8
"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=5.0)
    ap.add_argument("--parts", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    import trivy_amd._native as N
    import trivy_amd.secret as S
    dev = torch.device("cuda", 0)
    size = int(a.gb * 1e9)
    chunk = N.gen.tsg_gen_chunk_bytes()
    nch = (size + chunk - 1) // chunk
    ids = np.arange(nch, dtype=np.uint64)  # file 0, chunk k
    d_data = torch.zeros(size + 4096, dtype=torch.uint8, device=dev)
    d_off = torch.tensor([0, size + 1], dtype=torch.int64, device=dev)
    d_ids = torch.from_numpy(ids.view(np.int64)).to(dev)
    d_paths = torch.empty(64, dtype=torch.uint8, device=dev)
    d_poff = torch.empty(2, dtype=torch.int64, device=dev)
    cap = max(1 << 16, int(size * 1e-6 * 4) + 1024)
    rec = N.gen.tsg_gen_plant_record_size()
    d_pl = torch.empty(cap * rec, dtype=torch.uint8, device=dev)
    d_np = torch.zeros(1, dtype=torch.int64, device=dev)
    N.check(N.gen.tsg_gen_corpus_device(
        ctypes.c_void_p(d_data.data_ptr()), ctypes.c_void_p(d_off.data_ptr()), ctypes.c_void_p(d_ids.data_ptr()),
        nch, ctypes.c_void_p(d_paths.data_ptr()), ctypes.c_void_p(d_poff.data_ptr()), 1, 2024, 1e-6,
        ctypes.c_void_p(d_pl.data_ptr()), cap, ctypes.c_void_p(d_np.data_ptr())))
    torch.cuda.synchronize()
    del d_ids
    sc = S.new_scanner(None, device=0)
    eng = S.get_engine(0)
    rs = sc._rs.handle
    path = ctypes.c_char_p(b"logs/huge.log")
    d_path1 = torch.tensor(list(b"logs/huge.log"), dtype=torch.uint8, device=dev)
    d_poff1 = torch.tensor([0, len(b"logs/huge.log")], dtype=torch.int64, device=dev)
    base = d_data.data_ptr()

    def locs_of(res):
        n = N.lib.tsg_result_loc_count(res)
        p = N.lib.tsg_result_locs(res)
        return sorted((p[i].rule, p[i].start, p[i].end, p[i].start_line) for i in range(n))

    whole_stages = {}

    def whole():
        res = ctypes.c_void_p()
        t = time.perf_counter()
        N.check(N.lib.tsg_scan_device(eng, rs, ctypes.c_void_p(base), ctypes.c_void_p(d_off.data_ptr()),
                                      ctypes.c_void_p(d_path1.data_ptr()), ctypes.c_void_p(d_poff1.data_ptr()), 1,
                                      ctypes.byref(res)))
        dt = (time.perf_counter() - t) * 1e3
        out = locs_of(res)
        tm = (ctypes.c_double * 32)()
        nt = ctypes.c_size_t()
        N.lib.tsg_result_timings(res, tm, 32, ctypes.byref(nt))
        # (bench.py's stages_ms names; [15] the call's host wall, [16] its post-device part)
        names = ["path_gate", "scan_total", "expand", "sort_jobs", "verify", "exclude", "lines", "scan_kernels"]
        whole_stages.update({k: round(tm[i], 3) for i, k in enumerate(names)},
                            call_wall=round(tm[15], 3), post=round(tm[16], 3))
        N.lib.tsg_result_free(res)
        return dt, out

    from trivy_amd.shard import split_ranges
    halo = sc.part_halo()
    whole()  # warm-up (ruleset upload, buffers)
    w_ms = min(whole()[0] for _ in range(a.reps))
    _, want = whole()
    rows = []
    for W in a.parts:
        ranges = split_ranges(size, W, halo)
        best = None
        for _ in range(a.reps):
            part_ms, blobs = [], []
            for lo, hi, v0, v1 in ranges:
                b, n = ctypes.c_void_p(), ctypes.c_size_t()
                t = time.perf_counter()
                N.check(N.lib.tsg_scan_part_device(eng, rs, ctypes.c_void_p(base + v0), v0, v1 - v0, lo, hi, size, path,
                                                   ctypes.byref(b), ctypes.byref(n)))
                part_ms.append((time.perf_counter() - t) * 1e3)
                blobs.append((b, n.value))
            ptrs = (ctypes.c_void_p * W)(*[b for b, _ in blobs])
            lens = (ctypes.c_size_t * W)(*[n for _, n in blobs])
            res = ctypes.c_void_p()
            t = time.perf_counter()
            N.check(N.lib.tsg_scan_merge_device(eng, rs, ctypes.c_void_p(base), size, path, ptrs, lens, len(blobs),
                                                ctypes.byref(res)))
            m_ms = (time.perf_counter() - t) * 1e3
            got = locs_of(res)
            N.lib.tsg_result_free(res)
            part_bytes = sum(n for _, n in blobs)
            for b, _ in blobs:
                N.lib.tsg_part_free(b)
            assert got == want, f"split W={W}: {len(got)} locations vs {len(want)}"
            row = dict(parts=W, part_ms_max=round(max(part_ms), 3), part_ms_mean=round(sum(part_ms) / W, 3),
                       merge_ms=round(m_ms, 3), projected_ms=round(max(part_ms) + m_ms, 3),
                       part_blob_bytes=part_bytes, equal_locations=len(got))
            if best is None or row["projected_ms"] < best["projected_ms"]:
                best = row
        best["speedup_vs_whole"] = round(w_ms / best["projected_ms"], 2)
        rows.append(best)
    print(json.dumps(dict(tool="split_bench", file_gb=size / 1e9, whole_ms=round(w_ms, 3),
                          whole_gbps=round(size / w_ms / 1e6, 1), whole_stages_ms=whole_stages, findings=len(want),
                          splits=rows)))


if __name__ == "__main__":
    main()

"""Offline analysis of tools/gemv_lab's `tail` dump: where a GEMV launch's last microseconds go.

    ./tools/gemv_lab tail gpurun_out/gemv_tail.bin && python tools/gemv_tail.py gpurun_out/gemv_tail.bin

Per shape and rows-per-unit R: entry spread of the 4096 waves, staged/exit percentiles relative to the
launch's first entry, mean exit per XCD, and what the slowest 2 % of waves have in common (late entry,
XCD, wave slot in the workgroup, step count).
"""
import sys

import numpy as np

NAMES = ["qkv", "wo", "gu", "down"]


def main(path):
    raw = open(path, "rb").read()
    off = 0
    while off < len(raw):
        si, r, nl = np.frombuffer(raw, np.int32, 3, off)
        off += 12
        n = nl * 256 * 16 * 4
        st = np.frombuffer(raw, np.uint64, n, off).reshape(nl, 256 * 16, 4).astype(np.int64)
        off += n * 8
        st = st[2:]
        live = st[:, :, 3] != 0
        t0 = np.where(live, st[:, :, 0], np.iinfo(np.int64).max).min(axis=1, keepdims=True)
        ent = (st[:, :, 0] - t0) * 0.01
        stg = (st[:, :, 1] - t0) * 0.01
        ex = (st[:, :, 2] - t0) * 0.01
        steps = st[:, :, 3] & 0xFFFFFFFF
        xcd = (st[:, :, 3] >> 32) & 15
        pc = lambda a, q: float(np.percentile(a[live], q))
        name = NAMES[si % 100] + ("-i8" if si >= 100 else "")
        print(f"{name:8s} R{r}: entry p50 {pc(ent,50):5.2f} p99 {pc(ent,99):5.2f} max {pc(ent,100):5.2f} | "
              f"staged p50 {pc(stg,50):5.2f} p99 {pc(stg,99):5.2f} | exit p10 {pc(ex,10):5.2f} p50 {pc(ex,50):5.2f} "
              f"p90 {pc(ex,90):5.2f} p99 {pc(ex,99):5.2f} max {pc(ex,100):5.2f} us")
        print("      exit mean by XCD: " + " ".join(f"{x}:{ex[live & (xcd == x)].mean():5.2f}" for x in range(8)))
        run = ex - np.maximum(stg, 0)
        thr = np.percentile(ex[live], 98)
        slow = live & (ex >= thr)
        wslot = np.arange(256 * 16) % 16
        print(f"      slowest 2%: entry {ent[slow].mean():5.2f} (all {ent[live].mean():5.2f}), staged "
              f"{stg[slow].mean():5.2f} (all {stg[live].mean():5.2f}), run {run[slow].mean():5.2f} "
              f"(all {run[live].mean():5.2f}), steps {steps[slow].mean():6.1f} (all {steps[live].mean():6.1f})")
        print("      slowest 2% by XCD: " + " ".join(f"{x}:{int((slow & (xcd == x)).sum())}" for x in range(8))
              + " | by wave slot: " + " ".join(str(int((slow & (wslot[None, :] == w)).sum())) for w in range(16)))
        # what balancing would leave (round 6): per launch, the last wave's exit against the slowest workgroup's MEAN
        # wave exit (its waves sharing the workgroup's work) and the slowest XCD's mean (work shared per XCD)
        exm = np.where(live, ex, np.nan).reshape(ex.shape[0], -1, 16)
        end = np.nanmax(exm, axis=(1, 2))
        wg_mean = np.nanmax(np.nanmean(exm, axis=2), axis=1)
        xc = xcd.reshape(ex.shape[0], -1, 16)[:, :, 0]
        xcd_mean = np.nanmax(np.stack([np.nanmean(np.where(xc[:, :, None] == x, exm, np.nan), axis=(1, 2))
                                       for x in range(8)], axis=1), axis=1)
        print(f"      last exit p50 {np.median(end):5.2f} | slowest workgroup's mean exit p50 {np.median(wg_mean):5.2f} | "
              f"slowest XCD's mean exit p50 {np.median(xcd_mean):5.2f} | all-wave mean {np.nanmean(exm):5.2f} us")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/gemv_tail.bin")

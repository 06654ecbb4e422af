"""Diagnostic: dad_tail_ecda_w phase timeline (build variant 'stamps', -DDAD_PROBE_STAMPS; never the
product library).  Runs bench-shaped steps and prints the median phase ends (us after the tail
block's start) of the tail block and the four ECDA class blocks."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("DAD_LIB_VARIANT", "stamps")
import bench  # noqa: E402

PKG = bench.PKG
NB = 4   # class blocks of dad_tail_ecda_w (tail.hip TW_CB)


def main():
    B, T = 64, 300
    model = PKG.SSRLModel().cuda()
    P = bench.init_model_weights(model, seed=0)
    step = PKG.DADStep(model, flavor="iemocap", precision=os.environ.get("STAMP_PREC", "fp16"), rng="counter", seed=1)
    data = bench.make_batches(P, 2, B, T, seed=int(os.environ.get("STAMP_SEED", "17")), device=torch.device("cuda"),
                              random_labels=os.environ.get("STAMP_RANDLAB") == "1")
    S = 32  # slots per ECDA class (tail.hip ECDA_SLOTS)
    L = PKG.lib()
    reps = int(os.environ.get("STAMP_REPS", "15"))
    sleep = int(os.environ.get("STAMP_SLEEP", "0"))     # spin cycles queued ahead of each burst (0: none)
    store_fed = os.environ.get("STAMP_STORE") == "1"    # batches from store-mode loaders (tools/host_loader.py)
    if store_fed:
        n_utt = 1024
        g = torch.Generator(device="cuda")
        g.manual_seed(3)
        st = PKG.data.FeatureStore(torch.randn(n_utt * T, 768, device="cuda", generator=g), np.full(n_utt, T),
                                   np.arange(n_utt) * T, np.arange(n_utt) % 4, device=torch.device("cuda"))

        def epochs(loader):
            while True:
                yield from loader
        ci = epochs(PKG.data.DeviceLoader(st, batch_size=B, shuffle=True, fused=True))
        ni = epochs(PKG.data.DeviceLoader(st.subset(np.arange(n_utt), with_labels=False), batch_size=B, shuffle=True,
                                          fused=True))
        nxt = [(next(ci), next(ni))]
    raw = []
    for r in range(reps):   # the last step of a 4-step burst, reps times
        if sleep:
            torch.cuda._sleep(sleep)
        for i in range(4):   # (STAMP_AHEAD=1, the default: each step names the next, as the bench does)
            if store_fed:
                cur, nxt[0] = nxt[0], (next(ci), next(ni))
                step.step(cur[0], cur[1], 60, next_batch=nxt[0])
                continue
            nxt = data[(i + 1) % 2] if os.environ.get("STAMP_AHEAD", "1") == "1" else None
            step.step(data[i % 2][0], data[i % 2][1], 60, next_batch=nxt)
        torch.cuda.synchronize()
        ebuf = (ctypes.c_ulonglong * (NB * S + 16))()
        assert L.dad_probe_read_ecda_stamps(ebuf, len(ebuf)) == 0
        raw.append(np.frombuffer(ebuf, dtype=np.uint64).astype(np.int64))
    report_prep(read_prep_stamps(), raw[-1][NB * S])
    report(np.stack(raw[2:] if reps > 4 else raw))


def read_stamps():
    """The last tail launch's stamps (stamps build only)."""
    ebuf = (ctypes.c_ulonglong * (NB * 32 + 16))()
    assert PKG.lib().dad_probe_read_ecda_stamps(ebuf, len(ebuf)) == 0
    return np.frombuffer(ebuf, dtype=np.uint64).astype(np.int64)


def read_prep_stamps():
    """Per preparation wave (spare block xb, wave w -> index 8 xb + w): [start, end] wall clocks."""
    buf = (ctypes.c_ulonglong * (256 * 8 * 2))()
    assert PKG.lib().dad_probe_read_prep_stamps(buf, len(buf)) == 0
    return np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(256 * 8, 2)


def report_prep(ps, t0, nitems=192):
    """Preparation waves' start / end (us after the tail block's start), the waves that ran a
    pooling item first (block i mod nx, wave 0 for the first nx items) against the others."""
    ok = ps[:, 1] > 0
    idx = np.arange(len(ps))
    pool = ok & (idx % 8 == 0) & (idx // 8 < nitems)
    rest = ok & ~pool
    for name, m in (("pool waves", pool), ("other waves", rest)):
        if m.any():
            st, en = (ps[m, 0] - t0) / 100.0, (ps[m, 1] - t0) / 100.0
            print("prep %-11s n %4d  start med %.2f max %.2f  end med %.2f p90 %.2f max %.2f" % (
                name, m.sum(), np.median(st), st.max(), np.median(en), np.percentile(en, 90), en.max()))
    en = (ps[:, 1] - t0) / 100.0
    xcd = (idx // 8 + 1 + 4) % 8          # block id = xb + 1 + C, dispatched round-robin over the 8 XCDs
    print("prep end by XCD (median / max): " + "  ".join(
        "%d: %.1f/%.1f" % (x, np.median(en[ok & (xcd == x)]), en[ok & (xcd == x)].max()) for x in range(8)))
    print("prep end by wave slot (median / max): " + "  ".join(
        "%d: %.1f/%.1f" % (w, np.median(en[ok & (idx % 8 == w)]), en[ok & (idx % 8 == w)].max()) for w in range(8)))
    dur = (ps[:, 1] - ps[:, 0]) / 100.0
    print("prep duration (us): med %.2f p10 %.2f p90 %.2f max %.2f" % (
        np.median(dur[ok]), np.percentile(dur[ok], 10), np.percentile(dur[ok], 90), dur[ok].max()))
    late = ok & (en > np.percentile(en[ok], 95))
    print("latest 5%% waves by block: %s" % sorted(set((idx[late] // 8).tolist()))[:40])


def report(raw):
    S = 32
    T0 = NB * S
    t0 = raw[:, T0:T0 + 1]
    rel = np.nanmedian(np.where(raw > 0, (raw - t0) / 100.0, np.nan), axis=0)
    on = np.mean(raw > 0, axis=0) > 0.5
    print("class blocks stamped in %s of %d steps" % ([int(np.sum(raw[:, c * S] > 0)) for c in range(NB)], raw.shape[0]))
    print("median of %d steps; us after the tail block's start" % raw.shape[0])
    if on[T0 + 14]:
        ends = [rel[c * S + 8] for c in range(NB) if on[c * S + 8]]
        print("launch entry %.2f  tail block start 0  tail end %.2f  class ends %s  last preparation block end %s"
              % (rel[T0 + 14], rel[T0 + 1], " ".join("%.2f" % e for e in ends),
                 ("%.2f" % rel[T0 + 15]) if on[T0 + 15] else "-"))
    print("tail: " + "  ".join("%s %.2f" % (n, rel[T0 + k]) for k, n in ((4, "mask"), (2, "ce-wave"), (7, "certainty"), (8, "ranks"), (9, "quantile"),
                                                                          (10, "bcast"), (4, "dacp-wave"), (5, "kl"),
                                                                          (6, "w1-done"), (1, "end")) if on[T0 + k]))
    if on[T0 + 13] and on[T0 + 12]:
        ghz = np.median((raw[:, T0 + 13] - raw[:, T0 + 12]) / ((raw[:, T0 + 1] - raw[:, T0]) * 10.0))
        print("  tail block clock: %.2f GHz" % ghz)
    cyc = [(19, 13, "gates"), (13, 14, "stores+norm-math"), (14, 15, "norm-sums"), (15, 16, "zero+tables"),
           (16, 17, "centroid-partials"), (17, 18, "wsum")]
    for c in range(NB):
        o = c * S
        if all(on[o + a] and on[o + b] for a, b, _ in cyc):
            print("ecda class %d staging cycles: %s" % (c, "  ".join(
                "%s %d" % (n, int(np.median(raw[:, o + b] - raw[:, o + a]))) for a, b, n in cyc)))
    cyc2 = [(6, 20, "cent-dist"), (20, 21, "comp+bw"), (21, 22, "pairs"), (22, 23, "sums"), (23, 24, "b3+terms"),
            (24, 25, "mg-reads+mfma"), (25, 26, "mg-stage"), (26, 27, "mg-stores"), (27, 28, "flags")]
    for c in range(NB):
        o = c * S
        if not on[o + 20]:
            continue
        print("ecda class %d coef/grad cycles: %s" % (c, "  ".join(
            "%s %d" % (n, int(np.median(raw[:, o + b] - raw[:, o + a]))) for a, b, n in cyc2 if on[o + a] and on[o + b])))
    names = ["start", "dacp", "staged", "b1", "gram+cent", "b2", "b3", "b4", "end", "rows-landed", "", "", "cand-stored"]
    for c in range(NB):
        o = c * S
        if not on[o]:
            continue
        print("ecda class %d (cand %d, clean %d): %s" % (c, raw[-1, o + 10], raw[-1, o + 11], "  ".join(
            "%s %.2f" % (names[k], rel[o + k]) for k in (0, 1, 9, 12, 2, 3, 4, 5, 6, 7, 8) if on[o + k])))


if __name__ == "__main__":
    main()

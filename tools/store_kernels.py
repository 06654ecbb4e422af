"""Per-kernel times (HIP events, dad_timing_*) of the train step fed by resident padded batches and by
store-mode device loaders (bench.py data_path_bench's legs), each step naming the next batch as
train_epoch does, plus the wall time per step.   python tools/store_kernels.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

PKG = bench.PKG


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    PKG.lib()
    model = PKG.SSRLModel().to(dev)
    P = bench.init_model_weights(model, seed=0)
    view = PKG.ConfigView(None, flavor="iemocap")
    step = PKG.DADStep(model, view, precision="fp16", rng="counter", seed=1000)
    B, T, n_utt, epoch = 64, 300, 1024, 60
    # clean and noisy stores of the headline batches' distribution (STORE_RANDN=1: N(0, 1) features)
    if os.environ.get("STORE_RANDN") == "1":
        g = torch.Generator(device=dev)
        g.manual_seed(3)
        store = nstore = PKG.data.FeatureStore(torch.randn(n_utt * T, 768, device=dev, generator=g), np.full(n_utt, T),
                                               np.arange(n_utt) * T, np.arange(n_utt) % 4, device=dev)
    else:
        store = bench.synthetic_store(P, n_utt, T, dev, seed=3, noisy=False)
        nstore = bench.synthetic_store(P, n_utt, T, dev, seed=4, noisy=True)
    resident = bench.make_batches(P, 8, B, T, seed=17, device=dev)
    # the same store's utterances collated once into 8 resident padded batch pairs (store content,
    # padded addressing)
    rs = np.random.RandomState(5)
    collated = []
    for k in range(8):
        c = store.collate(rs.choice(n_utt, B, replace=False))
        nz = nstore.collate(rs.choice(n_utt, B, replace=False), with_labels=False)
        collated.append((c, nz))

    def epochs(loader):
        while True:
            yield from loader

    for mode in ("resident", "store", "collated", "resident", "store", "collated"):
        if mode == "store":
            ci = epochs(PKG.data.DeviceLoader(store, batch_size=B, shuffle=True, fused=True))
            ni = epochs(PKG.data.DeviceLoader(nstore.subset(np.arange(n_utt), with_labels=False), batch_size=B,
                                              shuffle=True, fused=True))
            src = lambda k: (next(ci), next(ni))  # noqa: E731
        elif mode == "collated":
            src = lambda k: collated[k % len(collated)]  # noqa: E731
        else:
            src = lambda k: resident[k % len(resident)][:2]  # noqa: E731
        nxt = [src(0)]

        def one(k):
            cur, nxt[0] = nxt[0], src(k + 1)
            step.step(cur[0], cur[1], epoch, next_batch=nxt[0])
        for k in range(8):
            one(k)
        torch.cuda.synchronize()
        n = 96
        timer = PKG._lib.KernelTimer(4, n // 4 + 1)
        t0 = time.perf_counter()
        for k in range(n):
            one(k)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        kt = timer.stop()
        print("%-9s wall %6.1f us/step (events on every 4th step)  %s" % (
            mode, dt * 1e6, "  ".join("%s %.1f" % (k, v[0] * 1e3) for k, v in kt.items())), flush=True)


if __name__ == "__main__":
    main()

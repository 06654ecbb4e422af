"""Host cost of the train step fed by device loaders (bench.py data_path_bench's legs): wall and
host-enqueue time per step for collating and store-mode loaders, then a cProfile of the store-mode
loop (top entries by own time).   python tools/host_loader.py"""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

PKG = bench.PKG


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    PKG.lib()
    model = PKG.SSRLModel().to(dev)
    bench.init_model_weights(model, seed=0)
    view = PKG.ConfigView(None, flavor="iemocap")
    step = PKG.DADStep(model, view, precision="fp16", rng="counter", seed=1000)
    B, T, n_utt, epoch = 64, 300, 1024, 60
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    store = PKG.data.FeatureStore(torch.randn(n_utt * T, 768, device=dev, generator=g), np.full(n_utt, T),
                                  np.arange(n_utt) * T, np.arange(n_utt) % 4, device=dev)

    def epochs(loader):
        while True:
            yield from loader

    for fused in (False, True, False, True):
        clean = PKG.data.DeviceLoader(store, batch_size=B, shuffle=True, fused=fused)
        noisy = PKG.data.DeviceLoader(store.subset(np.arange(n_utt), with_labels=False), batch_size=B,
                                      shuffle=True, fused=fused)
        ci, ni = epochs(clean), epochs(noisy)
        nxt = [(next(ci), next(ni))]

        def one():
            cur, nxt[0] = nxt[0], (next(ci), next(ni))
            step.step(cur[0], cur[1], epoch, next_batch=nxt[0])
        for _ in range(5):
            one()
        torch.cuda.synchronize()
        n = 64
        t0 = time.perf_counter()
        tl = 0.0
        for _ in range(n):
            a = time.perf_counter()
            cur, nxt[0] = nxt[0], (next(ci), next(ni))
            tl += time.perf_counter() - a
            step.step(cur[0], cur[1], epoch, next_batch=nxt[0])
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print("%-8s host %6.1f us/step (loaders %5.1f)  wall %6.1f us/step  prepped %s" %
              ("store" if fused else "collate", (t1 - t0) / n * 1e6, tl / n * 1e6, (t2 - t0) / n * 1e6,
               step.last_prepped), flush=True)
        if fused and os.environ.get("DAD_LIB_VARIANT") == "stamps":
            import tailw_stamps   # the last steps' tail-launch timelines, and the losses and range flag
            raw = []
            for _ in range(8):
                one()
                torch.cuda.synchronize()
                raw.append(tailw_stamps.read_stamps())
            tailw_stamps.report(np.stack(raw))
            print("losses", step.losses(), "range flag", step.decode_range_flag(step.range_flag()))
        if fused:
            pr = cProfile.Profile()
            pr.enable()
            for _ in range(64):
                one()
            pr.disable()
            torch.cuda.synchronize()
            s = io.StringIO()
            st = pstats.Stats(pr, stream=s)
            st.strip_dirs().sort_stats("tottime").print_stats(25)
            print(s.getvalue()[-6000:])
            break


if __name__ == "__main__":
    main()

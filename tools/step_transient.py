"""Diagnostic: per-step GPU time (events around every step) and host issue time in the first
timed steps after a short warm-up, as the driver's `bench.py --steps 20 --warmup 5` runs them.
Prints one line per segment."""
import sys, time
import torch
sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import bench

def main():
    warm = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    PKG = bench.PKG
    PKG.lib()
    model = PKG.SSRLModel().to(dev)
    P = bench.init_model_weights(model, seed=0)
    import argparse
    args = argparse.Namespace(flavor="iemocap", force_ecda=False, snr=5.0)
    view = bench.flavor_view(args)
    step = PKG.DADStep(model, view, precision="bf16", rng="counter", seed=1000, comm=None)
    data = bench.make_batches(P, bench.N_BATCHES, 64, 300, seed=17, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(warm):
        c, nb = data[i % len(data)]
        step.step(c, nb, 60)
    torch.cuda.synchronize()
    print("warm-up %d steps: %.2f ms" % (warm, (time.perf_counter() - t0) * 1e3))
    for seg in range(4):
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(21)]
        host = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(20):
            evs[i].record()
            h0 = time.perf_counter()
            c, nb = data[(warm + 20 * seg + i) % len(data)]
            step.step(c, nb, 60)
            host.append((time.perf_counter() - h0) * 1e6)
        evs[20].record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        gpu = [evs[i].elapsed_time(evs[i + 1]) * 1e3 for i in range(20)]
        print("seg %d: wall %.2f ms (%.1f us/step); gpu us/step %s; host us/step %s" % (
            seg, wall, wall * 50, " ".join("%.0f" % g for g in gpu), " ".join("%.0f" % h for h in host)))

main()

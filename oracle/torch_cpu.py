"""PyTorch-CPU restatement of the DAD train step: bench.py's CPU baseline (TEST/BENCH ONLY).

The NumPy oracle (dad_oracle.py) is the parity checker; it spells out an analytic backward
and runs ~2x slower than the reference on the same host.  This module is the CPU
*baseline*: the same step written against the same ATen operators the reference calls
(F.linear / addmm, randn_like, rand, randint, torch.quantile, autograd, clip_grad_norm_,
torch.optim.Adam), so its cost on a host is the reference's cost.  It is this repo's own
code -- the reference never travels to the GPU box -- and its step time is calibrated
against the imported reference in the build container (oracle/calibrate_cpu.py ->
profiles/r02_cpu_calibration.json, ratio ~1).

Step = the body of Trainer.train_epoch's loop (I/train.py:484-492): train_step
(I/train.py:397-471) + backward + clip_grad_norm_ + Adam + teacher EMA, for the IEMOCAP /
CASIA / EMODB switch resolution of dad_oracle.effective_switches.  Draws are torch's global
generator (the reference's behaviour), or injected (`draws=`) for the golden replay test.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from . import dad_oracle


class TorchCPUStep:
    def __init__(self, W1, b1, W2, b2, cfg, anchors=None):
        self.cfg = cfg
        mk = lambda a: torch.tensor(np.asarray(a, np.float32))
        self.student = [mk(a).requires_grad_(True) for a in (W1, b1, W2, b2)]
        self.teacher = [mk(a) for a in (W1, b1, W2, b2)]
        self.opt = torch.optim.Adam(self.student, lr=cfg["LEARNING_RATE"], weight_decay=cfg["WEIGHT_DECAY"])
        self.tau = torch.full((4,), 0.5)
        self.Q = torch.full((4,), 0.5)
        self.anchors = torch.zeros(4) if anchors is None else torch.as_tensor(anchors, dtype=torch.float32)
        self.score_lists = [[] for _ in range(4)]

    def load_state(self, st):
        """Seeded transition state (oracle/synth.make_state) -> params, Adam, DACP."""
        with torch.no_grad():
            for p, a in zip(self.student, st["student"]):
                p.copy_(torch.from_numpy(np.asarray(a, np.float32)))
            for p, a in zip(self.teacher, st["teacher"]):
                p.copy_(torch.from_numpy(np.asarray(a, np.float32)))
        for p, m, v in zip(self.student, st["exp_avg"], st["exp_avg_sq"]):
            self.opt.state[p] = {"step": torch.tensor(float(st["nstep"])), "exp_avg": torch.from_numpy(m.copy()),
                                 "exp_avg_sq": torch.from_numpy(v.copy())}
        self.tau = torch.from_numpy(np.asarray(st["tau"], np.float32).copy())
        self.Q = torch.from_numpy(np.asarray(st["Q"], np.float32).copy())

    # ------------------------------------------------------------------ model pieces
    @staticmethod
    def encode(x, pad, W1, b1):
        """masked mean of ReLU(x W1^T + b1) over the valid frames (I/model.py:18-41)"""
        h = torch.relu(F.linear(x, W1, b1))
        keep = (~pad).unsqueeze(-1).to(h.dtype)
        n = keep.sum(1).clamp(min=1.0)
        return (h * keep).sum(1) / n

    def classify(self, e, W2, b2, keep=None):
        """fc(dropout(e)) with the student's p (I/model.py:54-64)"""
        p = self.cfg["DROPOUT_RATE"]
        if keep is None:
            e = F.dropout(e, p, training=True)
        else:
            e = e * (torch.as_tensor(keep).to(e.dtype) / (1 - p))
        return F.linear(e, W2, b2)

    def augment(self, x, draws):
        """weak and strong augmentation (I/utils.py:328-375)"""
        c = self.cfg
        nw = torch.randn_like(x) if draws is None else torch.from_numpy(draws["nw"])
        weak = x + nw * c["WEAK_NOISE_STD"]
        ns = torch.randn_like(x) if draws is None else torch.from_numpy(draws["ns"])
        strong = x + ns * c["STRONG_NOISE_STD"]
        p = c["DROPOUT_RATE"]
        if p > 0:
            u = torch.rand(x.shape[-1]) if draws is None else torch.from_numpy(draws["u"])
            strong = strong * (u > p).float()
        B, T = x.shape[0], x.shape[1]
        mlen = int(T * c["TEMPORAL_MASK_RATIO"])
        if c["TEMPORAL_MASK_RATIO"] > 0 and mlen > 0:
            hi = max(1, T - mlen + 1)
            start = torch.randint(0, hi, (B,)) if draws is None else torch.from_numpy(np.asarray(draws["start"]))
            t = torch.arange(T)
            zero = (t[None, :] >= start[:, None]) & (t[None, :] < start[:, None] + mlen)
            strong = strong.masked_fill(zero.unsqueeze(-1), 0.0)
        return weak, strong

    def certainty(self, q, use_entropy):
        mx, pred = q.max(1)
        if not use_entropy:
            return mx, pred
        ent = -(q * torch.log2(q + 1e-8)).sum(1)
        return mx * (1 - ent / math.log2(q.shape[1])), pred

    def dacp(self, q, epoch, use_entropy):
        """DACPManager.calculate_mask (I/utils.py:449-507)"""
        c = self.cfg
        s, pred = self.certainty(q, use_entropy)
        w = torch.sigmoid(c["DACP_SENSITIVITY_K"] * (self.Q - self.Q.mean()))
        g = c["DACP_QUANTILE_START"] + (c["DACP_QUANTILE_END"] - c["DACP_QUANTILE_START"]) * (epoch / c["EPOCHS"])
        that = torch.stack([torch.quantile(s[pred == k], g) if bool((pred == k).any()) else self.tau[k]
                            for k in range(4)])
        floored = torch.max(that + c["DACP_CALIBRATION_STRENGTH_LAMBDA"] * (w - 0.5), self.anchors)
        a = c["DACP_THRESHOLD_SMOOTHING_ALPHA"]
        self.tau = a * self.tau + (1 - a) * floored
        mask = s >= self.tau[pred]
        for k in range(4):
            self.score_lists[k].extend(s[pred == k].detach().numpy())
        return mask, s, pred, w

    def ecda(self, ec, es, yc, pred, mask, s, w, class_aware):
        """ECDALoss.forward (I/utils.py:565-652)"""
        c = self.cfg
        if mask.dtype != torch.bool:
            mask = mask > c["FIXED_CONFIDENCE_THRESHOLD"]

        def mmd(Zs, Zt, ws, wt):
            Z = torch.cat([Zs, Zt])
            n = Z.shape[0]
            D = ((Z.unsqueeze(1) - Z.unsqueeze(0)) ** 2).sum(-1)
            bw = D.detach().sum() / (n * n - n) / 4.0
            K = sum(torch.exp(-D / (bw * 2 ** i + 1e-8)) for i in range(5))
            ns = Zs.shape[0]
            t = lambda blk, a, b: (blk * torch.outer(a, b)).sum() / (torch.outer(a, b).sum() + 1e-8)
            return t(K[:ns, :ns], ws, ws) + t(K[ns:, ns:], wt, wt) - 2 * t(K[:ns, ns:], ws, wt)

        total = torch.zeros(())
        if not class_aware:
            nz = es[mask]
            if ec.shape[0] >= 2 and nz.shape[0] >= 2:
                total = mmd(ec, nz, torch.ones(ec.shape[0]), torch.ones(nz.shape[0]))
            return total
        ncls = w.shape[0]
        cents = [es[(pred == k) & mask].mean(0) for k in range(ncls) if bool(((pred == k) & mask).any())]
        rep = -torch.pdist(torch.stack(cents)).mean() if len(cents) > 1 else torch.zeros(())
        att = torch.exp(c["ECDA_CLASS_ATTENTION_LAMBDA"] * (w.mean() - w))
        for k in range(ncls):
            zc = ec[yc == k]
            sel = (pred == k) & mask
            zt = es[sel]
            if zc.shape[0] < 2 or zt.shape[0] < 2:
                continue
            comp = ((zt - zt.mean(0)) ** 2).sum(1).mean()
            term = (mmd(zc, zt, torch.ones(zc.shape[0]), s[sel]) + c["ECDA_COMPACTNESS_WEIGHT_GAMMA"] * comp
                    + c["ECDA_REPULSION_WEIGHT_DELTA"] * rep)
            total = total + att[k] * term
        return total

    # ------------------------------------------------------------------------ step
    def step(self, inp, epoch, lr=None, draws=None):
        c = self.cfg
        use_dacp, use_ecda, use_entropy, class_aware = dad_oracle.effective_switches(c)
        w_kl, w_ecda, warm = dad_oracle.loss_weights(c, epoch)
        for g in self.opt.param_groups:
            g["lr"] = dad_oracle.cosine_lr(c, epoch) if lr is None else lr
        W1, b1, W2, b2 = self.student
        T1, Tb1, T2, Tb2 = self.teacher
        xc, mc = torch.from_numpy(inp["xc"]), torch.from_numpy(inp["mc"])
        yc = torch.from_numpy(inp["yc"])
        eps = c["LABEL_SMOOTHING_FACTOR"] if c["USE_LABEL_SMOOTHING"] else 0.0
        self.opt.zero_grad()
        ec = self.encode(xc, mc, W1, b1)
        zc = self.classify(ec, W2, b2, None if draws is None else draws["keep1"])
        ce = F.cross_entropy(zc, yc, label_smoothing=eps)
        out = {"e_clean": ec, "z_clean": zc}
        kl = torch.zeros(())
        ecda = torch.zeros(())
        total = ce
        if not warm:
            xn, mn = torch.from_numpy(inp["xn"]), torch.from_numpy(inp["mn"])
            weak, strong = self.augment(xn, draws)
            with torch.no_grad():
                q = F.softmax(F.linear(self.encode(weak, mn, T1, Tb1), T2, Tb2), dim=1)
            if use_dacp:
                mask, s, pred, w = self.dacp(q, epoch, use_entropy)
                maskf = mask.float()
            else:
                s, pred = q.max(1)
                maskf = (s >= c["FIXED_CONFIDENCE_THRESHOLD"]).float()
                mask, w = maskf, torch.ones_like(maskf)
            es = self.encode(strong, mn, W1, b1)
            zs = self.classify(es, W2, b2, None if draws is None else draws["keep2"])
            ls = F.log_softmax(zs, dim=1)
            if float(maskf.sum()) > 1:                  # I/train.py:444 (a host sync, as in the reference)
                klr = F.kl_div(ls, q, reduction="none").sum(1)
                kl = (klr * maskf).sum() / (maskf.sum() + 1e-8)
                if use_ecda and w_ecda > 0:
                    ecda = self.ecda(ec, es, yc, q.max(1)[1], mask, s, w, class_aware)
            total = ce + w_kl * kl + w_ecda * ecda
            out.update(z_strong=zs, mask=maskf)
        total.backward()
        if c["GRADIENT_CLIPPING"]:
            out["clip_norm"] = float(torch.nn.utils.clip_grad_norm_(self.student, c["MAX_GRAD_NORM"]))
        self.opt.step()
        if not warm:
            m = c["EMA_MOMENTUM"]
            with torch.no_grad():
                for t, s_ in zip(self.teacher, self.student):
                    t.mul_(m).add_(s_, alpha=1 - m)
        out.update(total_loss=float(total.detach()), supervised_ce_loss=float(ce.detach()),
                   consistency_loss=float(kl.detach()), ecda_loss=float(ecda.detach()))
        return out

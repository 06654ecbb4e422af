"""Host logic without a GPU: late-bound config resolution and the SSRLModel surface."""
import math
import types

import numpy as np
import pytest
import torch

import dadpkg
from oracle import dad_oracle

F32 = np.float32


@pytest.mark.parametrize("flavor", ["iemocap", "casia", "emodb"])
@pytest.mark.parametrize("epoch", [0, 29, 30, 35, 59, 60, 499])
def test_loss_weights_and_lr_match_oracle(flavor, epoch):
    p = dadpkg.pkg()
    view = p.ConfigView(flavor=flavor)
    ocfg = dad_oracle.make_cfg(flavor)
    assert view.loss_weights(epoch) == dad_oracle.loss_weights(ocfg, epoch)
    assert view.lr_at(epoch) == dad_oracle.cosine_lr(ocfg, epoch)
    assert view.effective_switches() == dad_oracle.effective_switches(ocfg)


def test_config_is_read_at_call_time():
    """Ablation runners mutate the config module between runs (I/run_granular_ablations.py:25-30)."""
    p = dadpkg.pkg()
    mod = types.ModuleType("config")
    mod.WEIGHT_ECDA = 0.3
    mod.USE_DACP = True
    view = p.ConfigView(mod)
    assert view.flavor == "iemocap"
    c1 = p.dad_config_for(view, 4, 20, 4, 20, 60, 1)
    mod.WEIGHT_ECDA = 0.5
    mod.USE_DACP = False
    c2 = p.dad_config_for(view, 4, 20, 4, 20, 60, 1)
    assert abs(c1.w_ecda - 0.3) < 1e-7 and abs(c2.w_ecda - 0.5) < 1e-7
    assert c1.use_dacp == 1 and c2.use_dacp == 0
    # EMODB ignores USE_DACP (E/train_emodb.py:419)
    emod = types.ModuleType("config_emodb")
    emod.USE_DACP = False
    assert p.ConfigView(emod).effective_switches()[0] is True


@pytest.mark.parametrize("flavor", ["iemocap", "casia", "emodb"])
def test_config_cache_keys_cover_every_read(flavor, monkeypatch):
    """ConfigCache keys a config on the CONFIG_KEYS values: every attribute dad_config_for reads
    from a view (over warm-up, ramp, ECDA start and late epochs, with and without an lr) is there."""
    p = dadpkg.pkg()
    C = p.config
    seen = set()
    orig = C.ConfigView.__getattr__

    def rec(self, name):
        seen.add(name)
        return orig(self, name)
    monkeypatch.setattr(C.ConfigView, "__getattr__", rec)
    view = C.ConfigView(flavor=flavor)
    for epoch in (0, 29, 30, 35, 59, 60, 499):
        for lr in (None, 1e-3):
            C.dad_config_for(view, 4, 20, 4, 20, epoch, 3, lr=lr)
    assert seen and seen <= set(C.CONFIG_KEYS), sorted(seen - set(C.CONFIG_KEYS))


def test_config_cache_is_byte_identical_and_follows_config_changes():
    """DADStep.make_config's ConfigCache: the same bytes as dad_config_for for every Adam step,
    counter, geometry, epoch and lr, and a changed config value (module source, overrides) is
    a new key, read at call time as dad_config_for reads it."""
    p = dadpkg.pkg()
    C = p.config
    mod = types.ModuleType("config")
    mod.WEIGHT_ECDA = 0.3
    view = C.ConfigView(mod)
    cache = C.ConfigCache()
    for args in [(64, 300, 64, 300, 60, None), (16, 40, 12, 50, 3, 1e-3), (16, 40, None, None, 1, None),
                 (64, 300, 64, 300, 35, None)]:
        Bc, Tc, Bn, Tn, epoch, lr = args
        for adam_step, counter in ((1, 0), (7, 123), (1000, 2 ** 40 + 5)):
            for prec in (0, 1, 2):
                kw = dict(lr=lr, precision=prec, rng_mode=1, seed=9, counter=counter)
                a = C.dad_config_for(view, Bc, Tc, Bn, Tn, epoch, adam_step, **kw)
                b = cache.config(view, Bc, Tc, Bn, Tn, epoch, adam_step, **kw)
                assert bytes(a) == bytes(b), (args, adam_step, counter, prec)
    mod.WEIGHT_ECDA = 0.5
    view.overrides["DROPOUT_RATE"] = 0.25
    a = C.dad_config_for(view, 64, 300, 64, 300, 60, 9, counter=4)
    b = cache.config(view, 64, 300, 64, 300, 60, 9, counter=4)
    assert bytes(a) == bytes(b) and abs(b.w_ecda - 0.5) < 1e-7 and abs(b.p_drop - 0.25) < 1e-7
    mod.LIST_VALUE = [1, 2]                         # unrelated attributes do not matter
    mod.WEAK_NOISE_STD = np.array(0.02)             # an unhashable value: computed without the cache
    a = C.dad_config_for(view, 64, 300, 64, 300, 60, 9, counter=4)
    assert bytes(a) == bytes(cache.config(view, 64, 300, 64, 300, 60, 9, counter=4))


def test_float32_scalars_follow_torch_semantics():
    p = dadpkg.pkg()
    c = p.dad_config_for(p.ConfigView(flavor="iemocap"), 64, 300, 64, 300, 60, 7)
    assert c.drop_scale == float(F32(1.0) / F32(0.9))                 # keep.div_(1-p)
    assert c.one_m_beta1 == float(F32(1 - 0.9))
    assert c.ema_one_m == float(F32(1.0 - 0.995))
    assert c.dacp_gamma == float(F32(0.4 + 0.4 * 60 / 500))
    assert c.mask_len == int(300 * 0.1) and c.start_hi == 300 - 30 + 1
    lr = 5e-4 * (1 + math.cos(math.pi * 60 / 500)) / 2
    assert c.lr_step_size == float(F32(lr / (1 - 0.9 ** 7)))
    assert c.bc2_sqrt == float(F32(math.sqrt(1 - 0.999 ** 7)))
    assert c.warmup == 0 and c.ecda_on == 1
    w = p.dad_config_for(p.ConfigView(flavor="casia"), 8, 20, 8, 20, 60, 1)
    assert w.use_dacp == 0 and w.ecda_on == 0 and abs(w.fixed_thr - 0.75) < 1e-7


def test_ssrl_model_surface():
    p = dadpkg.pkg()
    m = p.SSRLModel(types.SimpleNamespace(EMA_MOMENTUM=0.995))
    keys = ["student_encoder.pre_net.weight", "student_encoder.pre_net.bias",
            "student_classifier.fc_layer.weight", "student_classifier.fc_layer.bias",
            "teacher_encoder.pre_net.weight", "teacher_encoder.pre_net.bias",
            "teacher_classifier.fc_layer.weight", "teacher_classifier.fc_layer.bias"]
    assert list(m.state_dict().keys()) == keys                       # I/train.py:583, inference.py:183
    assert [n for n, _ in m.named_parameters()] == keys               # Adam/clip order
    assert sum(x.numel() for x in m.parameters()) == 395784
    assert sum(x.numel() for x in m.parameters() if x.requires_grad) == 197892
    assert m.ema_momentum == 0.995
    # parameters are views of the flat vectors; teacher initialised to the student
    w = m.student_encoder.pre_net.weight
    assert w.data_ptr() == m.student_flat.data_ptr()
    assert torch.equal(m.student_flat, m.teacher_flat)
    sd = {k: torch.randn_like(v) for k, v in m.state_dict().items()}
    m.load_state_dict(sd)
    assert torch.equal(m.student_flat[:256 * 768].view(256, 768), sd["student_encoder.pre_net.weight"])
    assert torch.equal(m.teacher_flat[-4:], sd["teacher_classifier.fc_layer.bias"])
    m2 = m.to(torch.float32)
    assert m2.student_encoder.pre_net.weight.data_ptr() == m2.student_flat.data_ptr()
    assert not m2.teacher_encoder.pre_net.weight.requires_grad


def test_pretrained_mapping(tmp_path):
    """pre_net.* -> encoder, post_net.* -> fc_layer (I/model.py:143-198); errors are swallowed."""
    p = dadpkg.pkg()
    ck = {"pre_net.weight": torch.randn(256, 768), "pre_net.bias": torch.randn(256),
          "post_net.weight": torch.randn(4, 256), "post_net.bias": torch.randn(4)}
    path = tmp_path / "best_model_fold_0.ckpt"
    torch.save(ck, path)
    cfg = types.SimpleNamespace(PRETRAINED_EMOTION2VEC_PATH=str(path))
    m = p.SSRLModel(cfg)
    assert torch.equal(m.student_encoder.pre_net.weight, ck["pre_net.weight"])
    assert torch.equal(m.teacher_classifier.fc_layer.bias, ck["post_net.bias"])
    m.load_complete_pretrained_weights(str(tmp_path / "missing.ckpt"))   # must not raise


def test_encoder_refuses_cpu_tensors():
    p = dadpkg.pkg()
    m = p.SSRLModel()
    with pytest.raises(RuntimeError):
        m.student_encoder(torch.zeros(2, 5, 768), torch.zeros(2, 5, dtype=torch.bool))

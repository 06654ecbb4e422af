"""Epoch-level state and checkpoint formats on the CPU (checkpoint.py, config.lr_at): the cosine
schedule against torch's own CosineAnnealingLR, the Adam state-dict format against
torch.optim.Adam, and loading a checkpoint in the reference's format (I/train.py:581-592)
through the weights-only unpickler."""
import numpy as np
import pytest
import torch

import dadpkg

PKG = dadpkg.pkg()
CK = PKG.checkpoint


@pytest.mark.parametrize("flavor", ["iemocap", "casia", "emodb"])
def test_lr_schedule_matches_torch_cosine_annealing(flavor):
    view = PKG.ConfigView(flavor=flavor)
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.Adam([p], lr=view.LEARNING_RATE)
    sch = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=view.EPOCHS)   # I/train.py:363
    for epoch in range(view.EPOCHS + 1):
        got = view.lr_at(epoch)
        ref = opt.param_groups[0]["lr"]
        assert got == pytest.approx(ref, rel=1e-9, abs=1e-15), epoch
        assert np.float32(got) == np.float32(ref) or abs(got - ref) < 1e-12
        opt.step()
        sch.step()


def _reference_optimizer(model, steps=2, seed=0):
    """A real torch Adam over SSRLModel.parameters() as the reference builds it (I/train.py:362),
    stepped with seeded gradients on the student's parameters only."""
    g = torch.Generator().manual_seed(seed)
    opt = torch.optim.Adam(model.parameters(), lr=5e-4, weight_decay=1e-5)
    stu = [p for n, p in model.named_parameters() if n.startswith("student")]
    for _ in range(steps):
        for p in stu:
            p.grad = torch.randn(p.shape, generator=g)
        opt.step()
    return opt


def test_adam_state_dict_round_trips_with_torch_adam():
    model = PKG.SSRLModel()
    opt = _reference_optimizer(model)
    sd = opt.state_dict()
    m, v, n, lr = CK.load_adam_state_dict(sd, "cpu")
    assert n == 2 and lr == 5e-4 and m.shape == (PKG._lib.DAD_NPARAM,)
    ours = CK.adam_state_dict(m, v, n, lr, 1e-5)
    assert ours["param_groups"][0].keys() == sd["param_groups"][0].keys()
    assert ours["param_groups"][0] == sd["param_groups"][0]
    assert ours["state"].keys() == sd["state"].keys()
    for i in sd["state"]:
        for k in ("step", "exp_avg", "exp_avg_sq"):
            assert torch.equal(ours["state"][i][k], sd["state"][i][k]), (i, k)
    fresh = torch.optim.Adam(PKG.SSRLModel().parameters(), lr=1.0)
    fresh.load_state_dict(ours)                 # the reference's optimizer accepts it
    assert fresh.param_groups[0]["lr"] == 5e-4


def test_reference_format_checkpoint_loads_weights_only(tmp_path):
    model = PKG.SSRLModel()
    opt = _reference_optimizer(model, steps=1, seed=3)
    res = {"accuracy": 50.0, "weighted_accuracy": 47.5, "confusion_matrix": np.arange(16).reshape(4, 4),
           "f1_per_class": [0.1, 0.2, 0.3, 0.4]}
    ck = {"epoch": 12, "model_state_dict": model.state_dict(), "optimizer_state_dict": opt.state_dict(),
          "clean_results": res, "noisy_results": res}
    path = str(tmp_path / "iemocap_cross_domain_best.pth")
    torch.save(ck, path)                        # exactly the reference's save_checkpoint dict
    target = PKG.SSRLModel()
    got = CK.load_checkpoint(path, target)
    assert got["epoch"] == 12
    np.testing.assert_array_equal(got["noisy_results"]["confusion_matrix"], np.arange(16).reshape(4, 4))
    for (n1, a), (n2, b) in zip(model.state_dict().items(), target.state_dict().items()):
        assert n1 == n2 and torch.equal(a, b)


def test_early_stopping_counts_epochs_without_improvement():
    es = CK.EarlyStopping(patience=3)
    assert [es(b) for b in (True, False, False, True, False, False, False)] == \
        [False, False, False, False, False, False, True]
    assert not CK.EarlyStopping(patience=1, enabled=False)(False)


def test_next_batch_prepared_ahead_only_when_device_resident():
    """a step prepares the named next batch only if its tensors are the ones the next
    step will use in place (step._resident / _draws_resident); a host batch would be copied twice.
    The predicates are device-generic, so the CPU plays the step's device here."""
    S = PKG.step
    cpu = torch.device("cpu")
    meta = torch.device("meta")

    def batch(x_dtype=torch.float32, m_dtype=torch.bool, y_dtype=torch.int64, dev=cpu):
        return {"net_input": {"feats": torch.zeros(2, 5, 768, dtype=x_dtype, device=dev),
                              "padding_mask": torch.zeros(2, 5, dtype=m_dtype, device=dev)},
                "labels": torch.zeros(2, dtype=y_dtype, device=dev)}

    assert S._resident(batch(), cpu)
    assert not S._resident(batch(), meta)                    # another device: would be copied
    assert not S._resident(batch(x_dtype=torch.float64), cpu)
    assert not S._resident(batch(m_dtype=torch.uint8), cpu)
    assert not S._resident(batch(y_dtype=torch.int32), cpu)
    assert S._resident(batch(y_dtype=torch.int32), cpu, labels=False)
    nm = batch()
    nm["net_input"]["padding_mask"] = None                   # a fresh zero mask per call: new pointer
    assert not S._resident(nm, cpu)
    nc = batch()
    nc["net_input"]["feats"] = torch.zeros(2, 768, 5).transpose(1, 2)
    assert not S._resident(nc, cpu)
    d = {"nw": torch.zeros(3), "ns": torch.zeros(3), "u": torch.zeros(3), "start": torch.zeros(2, dtype=torch.int64),
         "keep1": torch.zeros(4, dtype=torch.bool), "keep2": torch.zeros(4, dtype=torch.bool)}
    assert S._draws_resident(d, cpu)
    assert not S._draws_resident(None, cpu)
    assert not S._draws_resident(dict(d, nw=np.zeros(3, np.float32)), cpu)
    assert not S._draws_resident(dict(d, start=torch.zeros(2, dtype=torch.int32)), cpu)

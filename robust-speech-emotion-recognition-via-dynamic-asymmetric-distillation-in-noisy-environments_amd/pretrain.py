"""Clean supervised pre-training step on the fused DAD kernels.

  BaseModel               IP/model.py:4-21     pre_net 768->256, ReLU, masked mean, post_net 256->4
  train_one_epoch         IP/train_for_clean.py:393-420   CE (no smoothing) + Adam(L2) per batch
  best_model_fold_k.ckpt  IP/train_for_clean.py:258-259   {pre_net.*, post_net.*} state dict

BaseModel is the DAD student without dropout: the same encoder and classifier.  Its step is
the fused DAD step in warm-up (CE on the clean batch only, no noisy branch, no EMA, no DACP)
with label smoothing off, dropout 0 and no gradient clipping: one dad_step per batch, all on
device.  The weights live in the student half of an SSRLModel; `base_state_dict()` writes the
pre-trainer's checkpoint format, which SSRLModel.load_complete_pretrained_weights reads
(I/model.py:143-198).
"""
import torch

from .config import ConfigView
from .model import SSRLModel
from .step import DADStep


class PretrainStep:
    def __init__(self, model=None, lr=2e-4, weight_decay=1e-5, precision="fp32", device="cuda"):
        self.model = model if model is not None else SSRLModel().to(device)
        # IP/config.py:16-18 defaults; IP/train_for_clean.py:154-155 (Adam(L2), CrossEntropyLoss())
        self.view = ConfigView(flavor="iemocap", WARMUP_EPOCHS=1 << 30, USE_LABEL_SMOOTHING=False, DROPOUT_RATE=0.0,
                               GRADIENT_CLIPPING=False, LEARNING_RATE=lr, WEIGHT_DECAY=weight_decay,
                               LEARNING_RATE_SCHEDULER="none")
        self.dad = DADStep(self.model, self.view, precision=precision, rng="counter")
        self.lr = lr

    def step(self, batch, lr=None):
        """optimizer.zero_grad(); loss = CE(model(feats, mask), labels); backward; step
        (IP/train_for_clean.py:407-411).  Returns (loss, logits) on the device."""
        losses = self.dad.step(batch, None, 0, lr=self.lr if lr is None else lr)
        B = batch["net_input"]["padding_mask"].shape[0]
        return losses["supervised_ce_loss"], self.dad.outputs(B, 0)["z_clean"]

    def train_one_epoch(self, loader, lr=None):
        """IP/train_for_clean.py:393-420: (mean batch loss, accuracy); one host read at the end."""
        tot, correct, n, nb = None, None, 0, 0
        for batch in loader:
            loss, z = self.step(batch, lr)
            labels = batch["labels"].to(z.device)
            c = (torch.argmax(z, 1) == labels).sum()
            tot = loss.detach().clone() if tot is None else tot + loss
            correct = c if correct is None else correct + c
            n += labels.numel()
            nb += 1
        if nb == 0:
            return 0.0, 0.0
        return float(tot) / nb, float(correct) / n

    def base_state_dict(self):
        """BaseModel.state_dict() (the pre-trainer's best_model_fold_k.ckpt, IP/train_for_clean.py:258)."""
        m = self.model
        return {"pre_net.weight": m.student_encoder.pre_net.weight.detach().cpu().clone(),
                "pre_net.bias": m.student_encoder.pre_net.bias.detach().cpu().clone(),
                "post_net.weight": m.student_classifier.fc_layer.weight.detach().cpu().clone(),
                "post_net.bias": m.student_classifier.fc_layer.bias.detach().cpu().clone()}

    def load_base_state_dict(self, sd):
        m = self.model
        with torch.no_grad():
            m.student_encoder.pre_net.weight.copy_(sd["pre_net.weight"])
            m.student_encoder.pre_net.bias.copy_(sd["pre_net.bias"])
            m.student_classifier.fc_layer.weight.copy_(sd["post_net.weight"])
            m.student_classifier.fc_layer.bias.copy_(sd["post_net.bias"])
        self.dad.refresh_shadow()

"""`SSRLModel` drop-in (I/model.py:67-265) with the MI355X encoder underneath.

Same constructor (`SSRLModel(cfg)`), same sub-module names and state_dict keys
(`{student,teacher}_encoder.pre_net.{weight,bias}`,
`{student,teacher}_classifier.fc_layer.{weight,bias}`), same `parameters()` order.
Each network's four parameters are views into ONE flat device vector
[W1 | b1 | W2 | b2] (dad.h DAD_NPARAM), which is the layout the fused step kernels
update in place; `load_state_dict`, `.to()` and `.cuda()` keep the views intact.
"""
import torch
import torch.nn as nn

from . import _lib

H, D, C = 256, 768, 4
_SLICES = {
    "W1": (0, H * D, (H, D)),
    "b1": (H * D, H * D + H, (H,)),
    "W2": (H * D + H, H * D + H + C * H, (C, H)),
    "b2": (H * D + H + C * H, _lib.DAD_NPARAM, (C,)),
}


def _require_cuda(x, what):
    if not x.is_cuda:
        raise RuntimeError("%s: the MI355X-native encoder runs on the GPU only (got a %s tensor); "
                           "move the model and batch to 'cuda'" % (what, x.device))


class _EncoderFn(torch.autograd.Function):
    """HIP encoder forward (fused GEMM + bias + ReLU + masked mean pool) and its W1/b1 grads."""

    @staticmethod
    def forward(ctx, x, pad_u8, w1, b1, precision):
        B, T, _ = x.shape
        e = torch.empty(B, H, device=x.device, dtype=torch.float32)
        ws = torch.empty(int(_lib.lib().dad_encoder_workspace_bytes(B, T)), device=x.device, dtype=torch.uint8)
        st = torch.cuda.current_stream(x.device).cuda_stream
        _lib.check(_lib.lib().dad_encoder_forward(_lib.ptr(x), _lib.ptr(pad_u8), B, T, _lib.ptr(w1), _lib.ptr(b1),
                                                  _lib.ptr(e), int(precision), _lib.ptr(ws), st),
                   "dad_encoder_forward")
        ctx.save_for_backward(x, pad_u8, w1, b1)
        return e

    @staticmethod
    def backward(ctx, de):
        x, pad_u8, w1, b1 = ctx.saved_tensors
        B, T, _ = x.shape
        de = de.contiguous().float()
        dw1 = torch.empty_like(w1)
        db1 = torch.empty_like(b1)
        ws = torch.empty(int(_lib.lib().dad_encoder_workspace_bytes(B, T)), device=x.device, dtype=torch.uint8)
        st = torch.cuda.current_stream(x.device).cuda_stream
        _lib.check(_lib.lib().dad_encoder_backward(_lib.ptr(x), _lib.ptr(pad_u8), B, T, _lib.ptr(w1), _lib.ptr(b1),
                                                   _lib.ptr(de), _lib.ptr(dw1), _lib.ptr(db1), _lib.ptr(ws), st),
                   "dad_encoder_backward")
        return None, None, dw1, db1, None


class Emotion2VecEncoder(nn.Module):
    """`Emotion2VecEncoder` (I/model.py:6-41): masked mean of ReLU(pre_net(x)) over frames."""

    def __init__(self, input_dim=768, hidden_dim=256, pretrained_path=None):
        super().__init__()
        if input_dim != D or hidden_dim != H:
            raise ValueError("MI355X encoder kernels are built for 768 -> 256")
        self.pre_net = nn.Linear(in_features=input_dim, out_features=hidden_dim)
        self.activate = nn.ReLU()
        self.precision = _lib.PREC_FP32

    def forward(self, x, padding_mask=None):
        _require_cuda(x, "Emotion2VecEncoder")
        x = x.contiguous().float()
        B, T, _ = x.shape
        if padding_mask is None:
            pad = torch.zeros(B, T, dtype=torch.uint8, device=x.device)
        else:
            pad = padding_mask.to(device=x.device, dtype=torch.bool).contiguous().view(torch.uint8)
        return _EncoderFn.apply(x, pad, self.pre_net.weight, self.pre_net.bias, self.precision)


class EmotionClassifier(nn.Module):
    """`EmotionClassifier` (I/model.py:44-64): fc(dropout(x))."""

    def __init__(self, input_dim: int, num_classes: int, dropout_rate: float = 0.1):
        super().__init__()
        self.dropout = nn.Dropout(dropout_rate)
        self.fc_layer = nn.Linear(in_features=input_dim, out_features=num_classes)

    def forward(self, x):
        return self.fc_layer(self.dropout(x))


class SSRLModel(nn.Module):
    """Student + EMA teacher (I/model.py:67-141)."""

    def __init__(self, cfg=None):
        super().__init__()
        g = (lambda k, d: getattr(cfg, k, d)) if cfg is not None else (lambda k, d: d)
        input_dim, hidden_dim = g("INPUT_DIM", 768), g("HIDDEN_DIM", 256)
        num_classes, dropout_rate = g("NUM_CLASSES", 4), g("DROPOUT_RATE", 0.1)
        if num_classes != C:
            raise ValueError("MI355X kernels are built for NUM_CLASSES=4")
        pretrained_path = g("PRETRAINED_EMOTION2VEC_PATH", None)
        self.student_encoder = Emotion2VecEncoder(input_dim, hidden_dim)
        self.student_classifier = EmotionClassifier(hidden_dim, num_classes, dropout_rate)
        self.teacher_encoder = Emotion2VecEncoder(input_dim, hidden_dim)
        self.teacher_classifier = EmotionClassifier(hidden_dim, num_classes, dropout_rate=0.0)
        # flat [W1|b1|W2|b2] storage (non-persistent buffers: state_dict keys stay the reference's)
        self.register_buffer("_student_flat", torch.empty(_lib.DAD_NPARAM), persistent=False)
        self.register_buffer("_teacher_flat", torch.empty(_lib.DAD_NPARAM), persistent=False)
        with torch.no_grad():
            for flat, enc, cls in ((self._student_flat, self.student_encoder, self.student_classifier),
                                   (self._teacher_flat, self.teacher_encoder, self.teacher_classifier)):
                for name, p in zip(("W1", "b1", "W2", "b2"), self._plist(enc, cls)):
                    a, b, _ = _SLICES[name]
                    flat[a:b].copy_(p.detach().reshape(-1))
        self._bind_views()
        if pretrained_path:
            self.load_complete_pretrained_weights(pretrained_path)
        self._init_teacher_network()
        self.ema_momentum = g("EMA_MOMENTUM", 0.99)
        self.param_writes = 0      # parameter writes by kernels outside a DADStep (shadow refresh key)

    @staticmethod
    def _plist(enc, cls):
        return [enc.pre_net.weight, enc.pre_net.bias, cls.fc_layer.weight, cls.fc_layer.bias]

    def _bind_views(self):
        for flat, enc, cls in ((self._student_flat, self.student_encoder, self.student_classifier),
                               (self._teacher_flat, self.teacher_encoder, self.teacher_classifier)):
            mods = [(enc.pre_net, "weight"), (enc.pre_net, "bias"), (cls.fc_layer, "weight"), (cls.fc_layer, "bias")]
            for name, (mod, attr) in zip(("W1", "b1", "W2", "b2"), mods):
                a, b, shape = _SLICES[name]
                old = getattr(mod, attr)
                p = nn.Parameter(flat[a:b].view(shape), requires_grad=old.requires_grad)
                setattr(mod, attr, p)

    def _apply(self, fn, recurse=True):
        # move/cast the flat vectors once and re-bind every parameter as a view of them
        req = {n: p.requires_grad for n, p in self.named_parameters()}
        self._student_flat = fn(self._student_flat)
        self._teacher_flat = fn(self._teacher_flat)
        self._bind_views()
        for n, p in self.named_parameters():
            p.requires_grad_(req[n])
        return self

    @property
    def student_flat(self):
        return self._student_flat

    @property
    def teacher_flat(self):
        return self._teacher_flat

    def set_precision(self, precision):
        for enc in (self.student_encoder, self.teacher_encoder):
            enc.precision = precision

    def load_complete_pretrained_weights(self, pretrained_path):
        """Map a BaseModel state_dict (`pre_net.*`, `post_net.*`) onto the student
        (I/model.py:143-198); errors are reported and swallowed, as in the reference."""
        try:
            ckpt = torch.load(pretrained_path, map_location="cpu", weights_only=True)
            enc = {k: v for k, v in ckpt.items() if k.startswith("pre_net")}
            cls = {k.replace("post_net", "fc_layer"): v for k, v in ckpt.items() if k.startswith("post_net")}
            if enc:
                self.student_encoder.load_state_dict(enc, strict=False)
            if cls:
                self.student_classifier.load_state_dict(cls, strict=False)
            print("loaded pretrained weights: %d encoder + %d classifier tensors" % (len(enc), len(cls)))
        except Exception as e:   # reference behaviour: report and keep random init
            print("failed to load pretrained weights: %s" % e)

    def _init_teacher_network(self):
        """Teacher := student, frozen (I/model.py:200-209)."""
        with torch.no_grad():
            self._teacher_flat.copy_(self._student_flat)
        for p in list(self.teacher_encoder.parameters()) + list(self.teacher_classifier.parameters()):
            p.requires_grad = False

    @torch.no_grad()
    def update_teacher_ema(self):
        """teacher = teacher*m + student*(1-m) (I/model.py:211-223), one HIP launch."""
        _require_cuda(self._student_flat, "update_teacher_ema")
        m = float(self.ema_momentum)
        _lib.check(_lib.lib().dad_teacher_ema(_lib.ptr(self._student_flat), _lib.ptr(self._teacher_flat),
                                              _lib.DAD_NPARAM, float(torch.tensor(m).float()),
                                              float(torch.tensor(1.0 - m).float()),
                                              torch.cuda.current_stream(self._student_flat.device).cuda_stream),
                   "dad_teacher_ema")
        self.param_writes += 1

    def predict(self, x, padding_mask=None, use_teacher=False):
        """Eval-mode logits (I/model.py:225-245)."""
        self.eval()
        with torch.no_grad():
            if use_teacher:
                return self.teacher_classifier(self.teacher_encoder(x, padding_mask))
            return self.student_classifier(self.student_encoder(x, padding_mask))

    def get_embeddings(self, x, padding_mask=None, use_teacher=False):
        """Eval-mode encoder outputs (I/model.py:247-265)."""
        self.eval()
        with torch.no_grad():
            enc = self.teacher_encoder if use_teacher else self.student_encoder
            return enc(x, padding_mask)

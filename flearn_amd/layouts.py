"""state_dict layouts of the BASELINE configs, by shape arithmetic (torchvision is not installed).

Used to build synthetic uploads with the real key/shape structure (many small tensors plus a few
large ones, BN buffers, 0-d int64 counters) for benches and tests:

    lenet5      44,426 fp32 in 10 tensors                               (config 1)
    resnet18    11,699,112 fp32 in 102 tensors + 20 int64 0-d buffers    (configs 2, 4)
    resnet50    25,610,152 fp32 in 267 tensors + 53 int64 0-d buffers    (config 3)
    vit_b_16    86,567,656 fp32 in 152 tensors                           (config 5)
"""
from __future__ import annotations

import math

import numpy as np


def lenet5():
    return [
        ("conv1.weight", (6, 1, 5, 5), "f32"), ("conv1.bias", (6,), "f32"),
        ("conv2.weight", (16, 6, 5, 5), "f32"), ("conv2.bias", (16,), "f32"),
        ("fc1.weight", (120, 256), "f32"), ("fc1.bias", (120,), "f32"),
        ("fc2.weight", (84, 120), "f32"), ("fc2.bias", (84,), "f32"),
        ("fc3.weight", (10, 84), "f32"), ("fc3.bias", (10,), "f32"),
    ]


def _bn(prefix, c):
    return [
        (f"{prefix}.weight", (c,), "f32"), (f"{prefix}.bias", (c,), "f32"),
        (f"{prefix}.running_mean", (c,), "f32"), (f"{prefix}.running_var", (c,), "f32"),
        (f"{prefix}.num_batches_tracked", (), "i64"),
    ]


def _resnet(bottleneck: bool, blocks, num_classes=1000):
    L = [("conv1.weight", (64, 3, 7, 7), "f32")] + _bn("bn1", 64)
    inplanes, exp = 64, (4 if bottleneck else 1)
    for li, (planes, nb) in enumerate(zip((64, 128, 256, 512), blocks), start=1):
        for b in range(nb):
            p = f"layer{li}.{b}"
            stride2 = b == 0 and li > 1
            if bottleneck:
                L += [(f"{p}.conv1.weight", (planes, inplanes, 1, 1), "f32")] + _bn(f"{p}.bn1", planes)
                L += [(f"{p}.conv2.weight", (planes, planes, 3, 3), "f32")] + _bn(f"{p}.bn2", planes)
                L += [(f"{p}.conv3.weight", (planes * exp, planes, 1, 1), "f32")] + _bn(f"{p}.bn3", planes * exp)
            else:
                L += [(f"{p}.conv1.weight", (planes, inplanes, 3, 3), "f32")] + _bn(f"{p}.bn1", planes)
                L += [(f"{p}.conv2.weight", (planes, planes, 3, 3), "f32")] + _bn(f"{p}.bn2", planes)
            if b == 0 and (stride2 or inplanes != planes * exp):
                L += [(f"{p}.downsample.0.weight", (planes * exp, inplanes, 1, 1), "f32")]
                L += _bn(f"{p}.downsample.1", planes * exp)
            inplanes = planes * exp
    L += [("fc.weight", (num_classes, 512 * exp), "f32"), ("fc.bias", (num_classes,), "f32")]
    return L


def resnet18():
    return _resnet(False, (2, 2, 2, 2))


def resnet50():
    return _resnet(True, (3, 4, 6, 3))


def vit_b_16(num_classes=1000, d=768, layers=12, mlp=3072, patches=196):
    L = [("class_token", (1, 1, d), "f32"), ("conv_proj.weight", (d, 3, 16, 16), "f32"),
         ("conv_proj.bias", (d,), "f32"), ("encoder.pos_embedding", (1, patches + 1, d), "f32")]
    for i in range(layers):
        p = f"encoder.layers.encoder_layer_{i}"
        L += [
            (f"{p}.ln_1.weight", (d,), "f32"), (f"{p}.ln_1.bias", (d,), "f32"),
            (f"{p}.self_attention.in_proj_weight", (3 * d, d), "f32"),
            (f"{p}.self_attention.in_proj_bias", (3 * d,), "f32"),
            (f"{p}.self_attention.out_proj.weight", (d, d), "f32"),
            (f"{p}.self_attention.out_proj.bias", (d,), "f32"),
            (f"{p}.ln_2.weight", (d,), "f32"), (f"{p}.ln_2.bias", (d,), "f32"),
            (f"{p}.mlp.0.weight", (mlp, d), "f32"), (f"{p}.mlp.0.bias", (mlp,), "f32"),
            (f"{p}.mlp.3.weight", (d, mlp), "f32"), (f"{p}.mlp.3.bias", (d,), "f32"),
        ]
    L += [("encoder.ln.weight", (d,), "f32"), ("encoder.ln.bias", (d,), "f32"),
          ("heads.head.weight", (num_classes, d), "f32"), ("heads.head.bias", (num_classes,), "f32")]
    return L


LAYOUTS = {"lenet5": lenet5, "resnet18": resnet18, "resnet50": resnet50, "vit_b_16": vit_b_16}


def get(name):
    return LAYOUTS[name]()


def fp32_elems(layout) -> int:
    return sum(math.prod(s) for _, s, t in layout if t == "f32")


def fp32_tensors(layout) -> int:
    return sum(1 for _, _, t in layout if t == "f32")


def padded_f32_stride(layout, align=64) -> int:
    """Row length of the f32 bucket for this layout (bucket.py's ALIGN padding per key)."""
    return sum(-(-max(math.prod(s), 1) // align) * align for _, s, t in layout if t == "f32")


def synthetic_state_dict(layout, flat: np.ndarray, counter: int = 0):
    """Split one flat fp32 row into a state_dict with the layout's keys (views into `flat`);
    int64 buffers get `counter`."""
    out, off = {}, 0
    for k, s, t in layout:
        if t == "f32":
            n = math.prod(s)
            out[k] = flat[off : off + n].reshape(s)
            off += n
        else:
            out[k] = np.array(counter, dtype=np.int64).reshape(s)
    return out

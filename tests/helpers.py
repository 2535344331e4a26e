"""Harness helpers shared by the CPU and GPU tests (plain PyTorch / numpy restatements of the
reference's off-path helpers; not part of the product)."""
import numpy as np
import torch

DTYPES = {'f32': np.float32, 'f64': np.float64}
TORCH_DTYPES = {'f32': torch.float32, 'f64': torch.float64}


def mask_iou(lhs, rhs):
    """kaolin/metrics/render.py:18-40"""
    b = lhs.shape[0]
    mul = lhs * rhs
    add = lhs + rhs
    up = torch.sum(mul.reshape(b, -1), dim=1)
    down = torch.sum((add - mul).reshape(b, -1), dim=1)
    return 1.0 - torch.mean(up / (down + 1e-10))


def shifted_mask(face_idx):
    """test_dibr.py:176-179: the covered mask shifted left by 5 pixels."""
    mask = face_idx != -1
    return torch.nn.functional.pad(mask, (0, 5))[..., 5:]


def iou_grad_soft(soft, face_idx):
    """d mask_iou(soft, shifted(face_idx)) / d soft on CPU, like test_dibr.py:167-191."""
    s = torch.as_tensor(np.asarray(soft)).clone().requires_grad_(True)
    fi = torch.as_tensor(np.asarray(face_idx))
    loss = mask_iou(s, shifted_mask(fi))
    loss.backward()
    return s.grad.numpy()


def sphere(inputs, dname, flip):
    key = f'{dname}_flip{flip}'
    return {k: inputs[f'{k}_{key}'] for k in ('fvz', 'fvi', 'uvs', 'valid', 'normals_z')}

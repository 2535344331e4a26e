"""``mask_iou`` -- drop-in for kaolin/metrics/render.py:18-40.

The silhouette loss of the DIB-R training step (examples/tutorial/ian_dibr.py:264-265):
``1 - mean_b(sum(l * r) / (sum(l + r - l * r) + 1e-10))``.  Forward: one HIP pass over both masks
(per-view fp64 partial sums, ordered finish, no host sync); backward: one elementwise HIP pass
(kaolin_amd/csrc/kd_metrics.hip).  The sums are accumulated in fp64, so fp32 results agree with
the reference's fp32 reductions to their rounding error, not bit for bit.
"""
import torch
from torch.autograd import Function

from .. import _C

__all__ = ['mask_iou']


class MaskIouHip(Function):
    """torch.autograd.Function over kd_mask_iou_forward / kd_mask_iou_backward."""

    @staticmethod
    def forward(ctx, lhs_mask, rhs_mask):
        loss, stats, _ = _C.mask_iou_forward(lhs_mask, rhs_mask)
        ctx.save_for_backward(lhs_mask, rhs_mask, stats)
        return loss

    @staticmethod
    def backward(ctx, grad_loss):
        lhs, rhs, stats = ctx.saved_tensors
        gl, gr = _C.mask_iou_backward(grad_loss, lhs, rhs, stats, ctx.needs_input_grad[0],
                                      ctx.needs_input_grad[1])
        return gl, gr


def mask_iou(lhs_mask, rhs_mask):
    r"""Compute the Intersection over Union of two segmentation masks
    (kaolin/metrics/render.py:18-40).

    Args:
        lhs_mask (torch.Tensor): (batch_size, height, width), float32 or float64, on a GPU.
        rhs_mask (torch.Tensor): same shape.

    Returns:
        (torch.Tensor): the IoU loss, a scalar.
    """
    batch_size, height, width = lhs_mask.shape
    assert rhs_mask.shape == lhs_mask.shape
    return MaskIouHip.apply(lhs_mask, rhs_mask)

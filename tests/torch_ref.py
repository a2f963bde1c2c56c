"""Independent PyTorch-CPU float64 formulations of the hot-path ops.

Used only by tests to pin the C oracle (oracle/) -- an independent second
implementation, written from the layout spec rather than
from the reference's index loops:
  a row of an H x W x C map is laid out as col = h + w*H + c*H*W
  (cnsl-cu-kernels.cu:32, :257), so row.view(C, W, H).transpose(1, 2) = [C,H,W];
  kernel matrix row = c*kh*kw + kx*kh + ky (cnsl-cu-kernels.cu:26-30).
"""
import numpy as np
import torch
import torch.nn.functional as F


def to_chw(x, H, W, C):
    x = torch.as_tensor(np.asarray(x), dtype=torch.float64)
    return x.reshape(-1, C, W, H).transpose(2, 3)          # [N, C, H, W]


def from_chw(t):
    N, C, H, W = t.shape
    return t.transpose(2, 3).reshape(N, C * W * H).numpy()


def kernel_to_oihw(K, kh, kw, C, G):
    K = torch.as_tensor(np.asarray(K), dtype=torch.float64)
    # row = c*kh*kw + kx*kh + ky  ->  [C, kw, kh, G] -> [G, C, kh, kw]
    return K.reshape(C, kw, kh, G).permute(3, 0, 2, 1).contiguous()


def conv_fwd(x, K, b, H, W, C, kh, kw, G, pad_h=0, pad_w=0):
    xt = to_chw(x, H, W, C)
    w = kernel_to_oihw(K, kh, kw, C, G)
    y = F.conv2d(xt, w, padding=(pad_h, pad_w))
    if b is not None:
        y = y + torch.as_tensor(np.asarray(b), dtype=torch.float64).view(1, -1, 1, 1)
    return from_chw(y)


def conv_grads(x, K, dy, H, W, C, kh, kw, G, pad_h=0, pad_w=0):
    """Returns (dx, gW in kernel-matrix layout, gb) in float64."""
    xt = to_chw(x, H, W, C).requires_grad_(True)
    w = kernel_to_oihw(K, kh, kw, C, G).requires_grad_(True)
    y = F.conv2d(xt, w, padding=(pad_h, pad_w))
    oh, ow = y.shape[2], y.shape[3]
    dyt = to_chw(dy, oh, ow, G)
    y.backward(dyt)
    dx = from_chw(xt.grad)
    gw = w.grad.permute(1, 3, 2, 0).reshape(C * kw * kh, G).numpy()
    gb = dyt.sum(dim=(0, 2, 3)).numpy()
    return dx, gw, gb


def maxpool_fwd(x, H, W, C, ph, pw, pc):
    t = to_chw(x, H, W, C).unsqueeze(1)                   # [N,1,C,H,W]
    y = F.max_pool3d(t, kernel_size=(pc, ph, pw))
    return from_chw(y.squeeze(1))

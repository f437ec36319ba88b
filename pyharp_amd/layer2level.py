"""Layer -> level interpolation used to build ``temf`` for the Planck source.

Mirror of harp::layer2level (src/utils/layer2level.hpp:16-41,
src/utils/layer2level.cpp:7-79; stencil src/utils/interp.hpp:7-21) on torch
tensors (any device).  Input (..., nlyr) at layer centres, output
(..., nlyr+1) at interfaces, same ordering as the input.
"""

from __future__ import annotations

from dataclasses import dataclass

import torch

K2ND_ORDER = 2
K4TH_ORDER = 4
K_EXTRAPOLATE = 0
K_CONSTANT = 1


@dataclass
class Layer2LevelOptions:
    order: int = K4TH_ORDER
    logx: bool = False
    logy: bool = False
    blower: int = K_EXTRAPOLATE
    bupper: int = K_CONSTANT
    check_positivity: bool = True


def layer2level(var: torch.Tensor, options: Layer2LevelOptions | None = None) -> torch.Tensor:
    op = options or Layer2LevelOptions()
    nlyr = var.shape[-1]
    out = torch.zeros(var.shape[:-1] + (nlyr + 1,), dtype=var.dtype, device=var.device)
    if nlyr == 1:
        out[..., 0] = var[..., 0]
    elif op.blower == K_EXTRAPOLATE:
        out[..., 0] = (3.0 * var[..., 0] - var[..., 1]) / 2.0
    elif op.blower == K_CONSTANT:
        out[..., 0] = var[..., 0]
    else:
        raise RuntimeError("Unsupported boundary condition")
    if op.order == K4TH_ORDER:
        if nlyr > 1:
            out[..., 1] = (var[..., 0] + var[..., 1]) / 2.0
        if nlyr > 2:
            out[..., nlyr - 1] = (var[..., nlyr - 1] + var[..., nlyr - 2]) / 2.0
        if nlyr > 3:
            cm = torch.tensor([-1.0 / 12.0, 7.0 / 12.0, 7.0 / 12.0, -1.0 / 12.0],
                              dtype=var.dtype, device=var.device)
            out[..., 2:nlyr - 1] = var.unfold(-1, 4, 1) @ cm
    elif op.order == K2ND_ORDER:
        if nlyr > 1:
            out[..., 1:nlyr] = (var[..., :nlyr - 1] + var[..., 1:]) / 2.0
    else:
        raise RuntimeError("Unsupported interpolation order")
    if nlyr == 1:
        out[..., nlyr] = var[..., nlyr - 1]
    elif op.bupper == K_EXTRAPOLATE:
        out[..., nlyr] = (3.0 * var[..., nlyr - 1] - var[..., nlyr - 2]) / 2.0
    elif op.bupper == K_CONSTANT:
        out[..., nlyr] = var[..., nlyr - 1]
    else:
        raise RuntimeError("Unsupported boundary condition")
    if op.check_positivity and bool((out < 0).any()):
        raise RuntimeError("layer2level check failed")
    return out

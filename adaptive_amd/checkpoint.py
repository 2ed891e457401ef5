"""Checkpoint I/O in the reference's format.

The reference saves ``model.state_dict()`` with ``torch.save`` after every epoch under the name
``cider-%.4f_model-%d.pkl`` (``code_src/train.py:177-178``) and restores it with
``model.load_state_dict(torch.load(path))`` (``code_src/models/model_factory.py:15-16``,
``code_src/tools/utils.py:263-266``).  ``Encoder2Decoder`` here has the same state-dict keys and
shapes; loading always uses ``torch.load(weights_only=True)`` (tensors only, nothing executed from
the file).  A reference checkpoint's ResNet trunk keys (``encoder.resnet_conv.*``) are dropped by
``Encoder2Decoder.load_state_dict`` when the model runs on post-trunk features.

Direction matters for the trunk: the reference's module always has the trunk and loads strictly
(``model.load_state_dict(torch.load(...))``), so a file written from a trunk-less model (the
default ``Encoder2Decoder(cf)``) lacks the 930 ``encoder.resnet_conv.*`` tensors and loads there
only with ``strict=False``.  Models built with ``trunk=True`` (or ``save_checkpoint(...,
trunk_state=...)`` with a torchvision-layout trunk state dict) write complete files that the
reference loads strictly.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import torch


def checkpoint_name(cider: float, epoch: int) -> str:
    """``train.py:178``: ``'cider-%.4f_model-%d.pkl' % (cider, epoch)``."""
    return "cider-%.4f_model-%d.pkl" % (cider, epoch)


def save_checkpoint(model: torch.nn.Module, directory: str, cider: float, epoch: int,
                    trunk_state: Optional[Dict[str, torch.Tensor]] = None) -> str:
    """``train.py:177-178``: the state dict (all tensors moved to the CPU so the file loads on
    any host) under the reference's epoch file name; returns the path.  ``trunk_state``: the
    ResNet-152 trunk's state dict (torchvision child layout, ``adaptive_amd.trunk.resnet_conv``)
    written under ``encoder.resnet_conv.*`` when the model has no trunk of its own, so that the
    reference's strict ``load_state_dict`` accepts the file (module docstring)."""
    path = os.path.join(directory, checkpoint_name(cider, epoch))
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    if trunk_state is not None:
        if any(k.startswith("encoder.resnet_conv.") for k in sd):
            raise ValueError("the model already carries a trunk; trunk_state would overwrite it")
        sd.update({"encoder.resnet_conv." + k: v.detach().cpu() for k, v in trunk_state.items()})
    torch.save(sd, path)
    return path


def load_checkpoint(model: torch.nn.Module, path: str, strict: bool = True):
    """``model_factory.py:16``: ``model.load_state_dict(torch.load(path))`` — tensors are mapped
    onto the model's device; ``weights_only=True`` refuses anything but tensors and containers."""
    dev = next(model.parameters()).device
    sd = torch.load(path, map_location=dev, weights_only=True)
    return model.load_state_dict(sd, strict=strict)


def start_epoch(path: str) -> int:
    """``model_factory.py:17-20``: the epoch a resumed run starts at, parsed exactly as the
    reference does — ``int(name.split('-')[1].split('.')[0]) + 1`` of the file name — which
    expects ``<algo>-<epoch>.pkl`` names.  (On the reference's own ``cider-X_model-N.pkl`` names
    it yields ``int(X's integer part) + 1``; kept as is so resumed runs behave identically.)"""
    return int(path.split("/")[-1].split("-")[1].split(".")[0]) + 1

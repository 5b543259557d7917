"""Minimal stand-in for the parts of ``lightning.pytorch`` the reference modules use (Lightning is not a
dependency of this build; the training loop lives in arcweld.trainer).

LightningModule: nn.Module + save_hyperparameters / hparams / log / device / load_from_checkpoint.
``log`` never synchronises the host: values are kept as detached device tensors and read out by the trainer
when it reports (the reference logs ``loss.item()`` per micro-batch, transformer_decoder.py:175).
Checkpoints use the Lightning layout ({"state_dict", "hyper_parameters", ...}) and load with
``torch.load(weights_only=True)`` only.
"""
from __future__ import annotations

import inspect

import torch
from torch import nn


class AttributeDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


class LightningModule(nn.Module):
    def __init__(self):
        super().__init__()
        self._hparams = AttributeDict()
        self._logged = {}
        self.trainer = None

    # -------------------------------------------------------------- hyper-parameters
    def save_hyperparameters(self, *args, **kwargs):
        """Collect the __init__ arguments of every class in the MRO being constructed (like Lightning)."""
        frame = inspect.currentframe().f_back
        collected = {}
        while frame is not None:
            code = frame.f_code
            if code.co_name != "__init__" or frame.f_locals.get("self") is not self:
                break
            argnames = code.co_varnames[1:code.co_argcount + code.co_kwonlyargcount]
            local = {k: frame.f_locals[k] for k in argnames if k in frame.f_locals}
            for k, v in local.items():
                collected.setdefault(k, v)          # innermost frame first; outer frames fill the rest
            frame = frame.f_back
        # the outermost (most-derived) constructor's values win
        frame = inspect.currentframe().f_back
        while frame is not None and frame.f_code.co_name == "__init__" and frame.f_locals.get("self") is self:
            code = frame.f_code
            for k in code.co_varnames[1:code.co_argcount + code.co_kwonlyargcount]:
                if k in frame.f_locals:
                    collected[k] = frame.f_locals[k]
            frame = frame.f_back
        collected.update(kwargs)
        self._hparams.update({k: v for k, v in collected.items() if _plain(v)})

    @property
    def hparams(self):
        return self._hparams

    # -------------------------------------------------------------- logging (no host sync)
    def log(self, name, value, *args, **kwargs):
        if isinstance(value, torch.Tensor):
            value = value.detach()
        self._logged[name] = value

    @property
    def logged(self):
        return self._logged

    @property
    def device(self):
        for p in self.parameters():
            return p.device
        return torch.device("cpu")

    # -------------------------------------------------------------- checkpoints
    def checkpoint_dict(self):
        return {"state_dict": {k: v.detach().cpu() for k, v in self.state_dict().items()},
                "hyper_parameters": dict(self._hparams), "pytorch-lightning_version": "arcweld-amd"}

    def save_checkpoint(self, path):
        torch.save(self.checkpoint_dict(), path)

    @classmethod
    def load_from_checkpoint(cls, checkpoint_path, map_location=None, strict=True, **overrides):
        ckpt = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
        hp = dict(ckpt.get("hyper_parameters", {}))
        hp.update(overrides)
        sig = inspect.signature(cls.__init__)
        accepted = {k: v for k, v in hp.items() if k in sig.parameters}
        model = cls(**accepted)
        model.load_state_dict(ckpt["state_dict"], strict=strict)
        if map_location is not None:
            model.to(map_location)
        return model


def _plain(v):
    return isinstance(v, (int, float, bool, str, type(None), tuple, list))


class LightningDataModule:
    def prepare_data(self):
        pass

    def setup(self, stage=None):
        pass

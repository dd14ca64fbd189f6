"""LinearHead — same module, parameters and persistence format as
DRT/model/linear.py:12-39 (``linear.pt`` state dict + ``head_config.json``).
On the inference path its projection runs on the HIP GEMM
(model/encoder.linear_head); the nn.Linear stays the parameter holder."""
from __future__ import annotations

import json
import logging
import os

import torch
import torch.nn as nn
from torch import Tensor

logger = logging.getLogger(__name__)


class LinearHead(nn.Module):
    def __init__(self, input_dim: int = 768, output_dim: int = 768):
        super().__init__()
        self.linear = nn.Linear(input_dim, output_dim, bias=False)
        self.config = {"input_dim": input_dim, "output_dim": output_dim}

    def forward(self, rep: Tensor = None):
        return self.linear(rep)

    @classmethod
    def load(cls, ckpt_dir: str):
        logger.info(f"Loading linear head from {ckpt_dir}")
        with open(os.path.join(ckpt_dir, "head_config.json")) as f:
            config = json.load(f)
        model = cls(**config)
        model.load_state_dict(torch.load(os.path.join(ckpt_dir, "linear.pt"), map_location="cpu", weights_only=True))
        return model

    def save(self, save_path):
        torch.save(self.state_dict(), os.path.join(save_path, "linear.pt"))
        with open(os.path.join(save_path, "head_config.json"), "w") as f:
            json.dump(self.config, f, indent=4)

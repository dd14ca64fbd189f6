"""CPU: Trainer host logic that needs no GPU (optimizer / scheduler construction).

Reference: DRT/trainer/trainer.py:85-112 (_get_optimizer_and_scheduler).  The LR schedulers are the
user's own DRT.trainer.scheduler classes (out of scope here); without that package a scheduler name
must fail with an error that names it, and no scheduler must still build the optimizer."""
import importlib.util
from types import SimpleNamespace

import pytest
import torch


def _bare_trainer(**args):
    from denseretrievaltoolkits_amd.trainer.trainer import Trainer
    tr = object.__new__(Trainer)
    tr.training_args = SimpleNamespace(learning_rate=1e-3, optimizer="adamw", **args)
    tr.model = torch.nn.Linear(4, 2)
    return tr


def test_optimizer_without_scheduler():
    tr = _bare_trainer(scheduler=None)
    tr._get_optimizer_and_scheduler()
    assert isinstance(tr.optimizer, torch.optim.AdamW)
    assert tr.optimizer.param_groups[0]["lr"] == 1e-3


@pytest.mark.skipif(importlib.util.find_spec("DRT") is not None, reason="the reference package is importable here")
def test_scheduler_without_reference_package_names_the_dependency():
    tr = _bare_trainer(scheduler="linear")
    with pytest.raises(ImportError, match="DRT.trainer.scheduler"):
        tr._get_optimizer_and_scheduler()

"""Training step of the TencentGR script on the grk path (model/BaseLine/main.py:163-190;
model/BaseLineO1/main.py:200-250): forward, loss, backward, optimizer -- with
no host synchronisation inside the step (the reference's ``np.where`` index
set and ``loss.item()`` are replaced by device-side counts)."""
from __future__ import annotations

import contextlib

import torch

from . import functional as G


class Trainer:
    """``step(batch)`` = one training step on a tensorised batch
    (``MyDataset.collate_tensor_fn`` layout, tensors on the device).

    loss: "bce" -- the reference loss (pos/neg BCE, main.py:177-182);
          "sampled_softmax" -- north-star in-batch sampled softmax.
    """

    def __init__(self, model, optimizer, loss='bce', amp_dtype=torch.bfloat16, temperature=0.05):
        if loss not in ('bce', 'sampled_softmax'):
            raise ValueError("loss must be 'bce' or 'sampled_softmax'")
        self.model, self.opt, self.loss_kind = model, optimizer, loss
        self.amp_dtype, self.temperature = amp_dtype, temperature

    def compute_loss(self, batch):
        seq, pos, neg, tt, ntt, _nat, sf, pf, nf = batch
        amp = (torch.autocast('cuda', dtype=self.amp_dtype) if self.amp_dtype is not None
               else contextlib.nullcontext())
        with amp:
            h, pe, ne = self.model.encode(seq, pos, neg, tt, sf, pf, nf)
            if self.loss_kind == 'bce':
                return G.bce_loss(h, pe, ne, ntt)
            return G.sampled_softmax_loss(h, pe, pos, ntt, self.temperature)

    def step(self, batch):
        self.opt.zero_grad()
        if hasattr(self.opt, 'prepare'):  # row-sharded tables: fetch this batch's rows from their owners
            self.opt.prepare(batch)
        if hasattr(self.opt, 'begin_step'):  # deferred table updates: bring this batch's rows up to date
            self.opt.begin_step(batch)
        loss = self.compute_loss(batch)
        loss.backward()
        self.opt.step()
        return loss.detach()

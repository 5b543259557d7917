"""Autoencoder base -- drop-in for model/autencoder_lightning_base.py:8-124 of the reference.

Same constructor, hyper-parameters, step methods, log keys and optimizer semantics; the loss arithmetic runs on
the HIP kernels (arcweld.functional) and the optimizer is the flat multi-tensor RAdam (arcweld.optim).
"""
from abc import abstractmethod

import torch
from torch import nn

from arcweld.functional import add_scalars, mse_loss
from arcweld.lightning import LightningModule
from arcweld.optim import RAdam


class Autoencoder(LightningModule):

    def __init__(self, hidden_dim: int, input_dim: int, num_embeddings: int, embedding_dim: int, n_resblocks: int,
                 learning_rate: float, seq_len: int = 200, dropout_p: float = 0.1):
        super().__init__()
        self.learning_rate = learning_rate
        self.dropout_p = dropout_p
        self.n_resblocks = n_resblocks
        self.num_embeddings: int = num_embeddings
        self.embedding_dim = embedding_dim
        self.hidden_dim = hidden_dim
        self.input_dim = input_dim
        self.seq_len = seq_len
        self.last_recon = (0, 0)
        # present in the reference but unused by its optimizer (autencoder_lightning_base.py:38-39, 122-124)
        self.betas = (0.9, 0.95)
        self.weight_decay = 0.1
        self.save_hyperparameters()

    @abstractmethod
    def forward(self, x: torch.Tensor):
        raise NotImplementedError

    def loss(self, preds: torch.Tensor, labels: torch.Tensor):
        return mse_loss(preds, labels)

    @staticmethod
    def weights_init(m):
        """Xavier-uniform weights and zero bias on every module whose class name contains 'Conv' (ref :70-78)."""
        classname = m.__class__.__name__
        if classname.find('Conv') != -1:
            try:
                nn.init.xavier_uniform_(m.weight.data)
                m.bias.data.fill_(0)
            except AttributeError:
                print("Skipping initialization of ", classname)

    def _forward_setp(self, x: torch.Tensor):
        embedding_loss, data_recon, perplexity = self(x)
        recon_error = mse_loss(data_recon, x)
        loss = add_scalars(recon_error, embedding_loss)
        return loss, recon_error, data_recon

    def training_step(self, batch, batch_idx):
        loss, recon_error, data_recon = self._forward_setp(batch)
        self.log('train/loss', loss, prog_bar=True)
        self.log('train/recon_error', recon_error)
        self.last_recon = (batch[:1].detach(), data_recon[:1].detach())
        return {'loss': loss, 'recon_error': recon_error}

    def validation_step(self, batch, batch_idx):
        loss, recon_error, data_recon = self._forward_setp(batch)
        self.log('val/loss', loss, sync_dist=True, on_epoch=True, prog_bar=True)
        self.log('val/recon_error', recon_error, sync_dist=True, on_epoch=True)
        return {'loss': loss, 'recon_error': recon_error, 'data_recon': data_recon}

    def test_step(self, batch, batch_idx):
        loss, recon_error, data_recon = self._forward_setp(batch)
        self.log('test/loss', loss, sync_dist=True, on_epoch=True, prog_bar=True)
        self.log('test/recon_error', recon_error, sync_dist=True, on_epoch=True)
        return {'loss': loss, 'recon_error': recon_error, 'data_recon': data_recon}

    def configure_optimizers(self):
        return RAdam(self.parameters(), lr=self.learning_rate)

"""VQ-VAE-Patch reconstruction training -- drop-in for the reference's train_reconstruction_embedding.py
(same flags, model construction, Trainer(gradient_clip_val, early stopping on val/loss, best/last checkpoints),
final test).  Data: ``--data-dir`` reads the reference's ASIMoW CSV (``<dir>/processed_asimow_dataset.csv``,
split by the reference's val/test (experiment, welding_run) ids, per-channel scaled; arcweld.asimow), or
``--data-npz`` an .npz with 'train'/'val'/'test' arrays of shape (n, 200, 2); without either the windows are
synthetic N(0, 1) 200x2 (the dataset is not available offline).  The W&B / MLflow loggers are not available
(CSVLogger only).  ``--precision`` picks the MFMA operand dtype: fp32 (default, the reference's numerics) or bf16
(opt-in, fp32 accumulation; arcweld.precision).
"""
import argparse
import logging as log
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from arcweld.data import ReconstructionDataModule  # noqa: E402
from arcweld.launch import CSVLogger, init_distributed, shutdown  # noqa: E402
from arcweld.precision import set_operand_dtype  # noqa: E402
from arcweld.trainer import EarlyStopping, ModelCheckpoint, Trainer  # noqa: E402
from model.vq_vae_patch_embedd import VQVAEPatch  # noqa: E402


def load_windows(path, device):
    with np.load(path, allow_pickle=False) as f:
        return tuple(torch.tensor(f[k], dtype=torch.float32, device=device) for k in ("train", "val", "test"))


def main(hparams):
    if hparams.use_wandb or hparams.use_mlflow:
        raise SystemExit("W&B / MLflow logging is not available in this build (no network); use the CSV logger")
    set_operand_dtype(hparams.precision)
    rank, world, dev = init_distributed()
    logger = CSVLogger("logs", name="vq-vae")
    logger.log_hyperparams({"model_name": hparams.model_name, "clipping_value": hparams.clipping_value,
                            **vars(hparams)})
    data = load_windows(hparams.data_npz, dev) if hparams.data_npz else None
    if hparams.data_dir:
        from arcweld import asimow
        ids = asimow.REFERENCE_SPLIT_IDS
        ds = asimow.load(hparams.data_dir, ids["val_ids"], ids["test_ids"], task="reconstruction", seed=hparams.seed)
        data = tuple(ds.tensors(s, device=dev)[0] for s in ("train", "val", "test"))
    data_module = ReconstructionDataModule(batch_size=hparams.batch_size, n_train=hparams.n_train,
                                           n_val=hparams.n_val, n_test=hparams.n_test, seed=hparams.seed,
                                           device=dev, data=data)
    data_module.setup(stage="fit")
    log.info(f"Loaded Data - Train dataset size: {len(data_module.train_ds)}")

    if hparams.model_name != "VQ-VAE-Patch":
        raise ValueError("Invalid model name")
    torch.manual_seed(hparams.seed)
    model = VQVAEPatch(hidden_dim=hparams.hidden_dim, input_dim=2, num_embeddings=hparams.num_embeddings,
                       embedding_dim=hparams.embedding_dim, n_resblocks=hparams.n_resblocks,
                       learning_rate=hparams.learning_rate, dropout_p=hparams.dropout_p,
                       patch_size=hparams.patch_size, batch_norm=bool(hparams.batchnorm),
                       use_improved_vq=bool(hparams.use_improved_vq), kmeans_iters=hparams.kmeans_iters,
                       threshold_ema_dead_code=hparams.threshold_ema_dead_code).to(dev)

    name = hparams.model_name
    checkpoint_callback = ModelCheckpoint(dirpath=f"model_checkpoints/{name}/", monitor="val/loss", mode="min",
                                          filename=f"{name}-best", save_last=True)
    early_stop_callback = EarlyStopping(monitor="val/loss", min_delta=0.0001, patience=5, verbose=False, mode="min")
    trainer = Trainer(devices=world, num_nodes=1, max_epochs=hparams.epochs, logger=logger,
                      callbacks=[checkpoint_callback, early_stop_callback], gradient_clip_val=hparams.clipping_value)
    trainer.fit(model=model, datamodule=data_module)
    trainer = Trainer(devices=1, num_nodes=1, logger=logger, callbacks=[checkpoint_callback])
    res = trainer.test(model=model, datamodule=data_module)
    if rank == 0:
        print("test:", res[0])
    shutdown()
    return res


def parser():
    p = argparse.ArgumentParser(description='Train VQ-VAE')
    p.add_argument('--epochs', type=int, help='Number of epochs to train', default=50)
    p.add_argument('--batch-size', type=int, help='Batch size', default=1024)
    p.add_argument('--num-embeddings', type=int, help='Number of embeddings', default=256)
    p.add_argument('--embedding-dim', type=int, help='Dimension of one embedding', default=32)
    p.add_argument('--hidden-dim', type=int, help='Hidden dimension', default=512)
    p.add_argument('--learning-rate', type=float, help='Learning rate', default=0.001)
    p.add_argument('--clipping-value', type=float, help='Gradient Clipping', default=0.7)
    p.add_argument('--n-resblocks', type=int, help='Number of Residual Blocks', default=8)
    p.add_argument('--patch-size', type=int, help='Patch size of the VQ-VAE Encoder', default=25)
    p.add_argument('--dropout-p', type=float, help='Dropout probability', default=0.1)
    p.add_argument('--batchnorm', type=int, help='Use the batch normalization layers', default=0)
    p.add_argument('--use-improved-vq', help='Use the improved VQ mechanism', action=argparse.BooleanOptionalAction)
    p.add_argument('--kmeans-iters', type=int, help='Number of K-Means iterations', default=10)
    p.add_argument('--threshold-ema-dead-code', type=int, help='Threshold for EMA dead code', default=2)
    p.add_argument('--model-name', type=str, help='Model name', default="VQ-VAE-Patch")
    p.add_argument('--use-wandb', action=argparse.BooleanOptionalAction)
    p.add_argument('--use-mlflow', action=argparse.BooleanOptionalAction)
    p.add_argument('--mlflow-url', type=str, default='')
    p.add_argument('--logging-entity', type=str)
    p.add_argument('--logging-project', type=str, default="asimow-vq-vae")
    # data source (this build): synthetic windows or an .npz of real windows
    p.add_argument('--data-npz', type=str, default="")
    p.add_argument('--data-dir', type=str, default="", help="directory holding processed_asimow_dataset.csv")
    p.add_argument('--n-train', type=int, default=8192)
    p.add_argument('--n-val', type=int, default=1024)
    p.add_argument('--n-test', type=int, default=1024)
    p.add_argument('--seed', type=int, default=0)
    p.add_argument('--precision', choices=["fp32", "bf16"], default="fp32",
                   help="MFMA operand dtype (bf16: opt-in, fp32 accumulation and master weights)")
    return p


if __name__ == '__main__':
    args = parser().parse_args()
    log.basicConfig(level=log.INFO, format='%(asctime)s - %(levelname)s - %(message)s')
    torch.set_float32_matmul_precision('medium')
    main(args)

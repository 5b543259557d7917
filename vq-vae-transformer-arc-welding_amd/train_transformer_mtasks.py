"""Latent-Transformer multi-task training -- drop-in for the reference's train_transformer_mtasks.py.

Same flags and stage loop: epoch_iter x (10 generation epochs, class_epoch classification epochs), the last
iteration replaced by classification fine-tuning (early stopping on val/cl/f1_score) and test; a new Trainer --
and so a new RAdam -- per stage; gradient_clip_val 0.8, accumulate_grad_batches 5; DDP over all GPUs with
``--use-all-gpus`` (launch with ``python -m torch.distributed.run --nproc-per-node N``).

Data: the frozen VQ-VAE (``--vqvae-model``: a checkpoint written by train_reconstruction_embedding.py; a
randomly initialised 512x64 VQ-VAE if the path does not exist) tokenizes synthetic welding sequences of n_cycles
200x2 windows on the GPU (arcweld.tokenize); ``--data-npz`` may provide real windows ('train'/'val'/'test' of
shape (n, n_cycles*200, 2) and '<split>_labels').  W&B / MLflow are not available (CSVLogger only).
``--precision`` picks the MFMA operand dtype (fp32 default, bf16 opt-in; arcweld.precision).  Without
``--use-all-gpus`` no process group is created (the reference trains on devices=1 then), even under torchrun.
"""
import argparse
import logging as log
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from arcweld.data import LatentPredDataModule, synthetic_labels, synthetic_windows  # noqa: E402
from arcweld.launch import CSVLogger, init_distributed, shutdown  # noqa: E402
from arcweld.precision import set_operand_dtype  # noqa: E402
from arcweld.trainer import EarlyStopping, Trainer  # noqa: E402
from model.transformer_decoder import MyTransformerDecoder  # noqa: E402
from model.vq_vae_patch_embedd import VQVAEPatch  # noqa: E402


def get_new_trainer(epochs_steps, logger, n_gpus=1):
    return Trainer(devices=n_gpus, num_nodes=1, max_epochs=epochs_steps, logger=logger, callbacks=[],
                   gradient_clip_val=0.8, accumulate_grad_batches=5)


def load_vqvae(path, dev):
    if path and os.path.exists(path):
        m = VQVAEPatch.load_from_checkpoint(path)
    else:
        log.warning(f"VQ-VAE checkpoint {path!r} not found: using a randomly initialised VQ-VAE-Patch "
                    "(H512, 8 ResBlocks, codebook 512x64, patch 25)")
        torch.manual_seed(1)
        m = VQVAEPatch(hidden_dim=512, input_dim=2, num_embeddings=512, embedding_dim=64, n_resblocks=8,
                       learning_rate=1e-3, dropout_p=0.1, patch_size=25, batch_norm=False)
    return m.to(dev).eval()


def load_splits(hparams, dev):
    if hparams.data_npz:
        with np.load(hparams.data_npz, allow_pickle=False) as f:
            return [(torch.tensor(f[k], dtype=torch.float32, device=dev),
                     torch.tensor(f[k + "_labels"], dtype=torch.long, device=dev)) for k in ("train", "val", "test")]
    sizes = (hparams.n_train, hparams.n_val, hparams.n_test)
    return [(synthetic_windows(n, hparams.n_cycles, hparams.seed + 11 * i, dev),
             synthetic_labels(n, hparams.seed + 11 * i, dev)) for i, n in enumerate(sizes)]


def load_dataset(hparams, dev, only_classify=False):
    vqvae = load_vqvae(hparams.vqvae_model, dev)
    splits = load_splits(hparams, dev)
    cls_dm = LatentPredDataModule(vqvae, splits, hparams.batch_size, task="autoregressive_ids_classification",
                                  seed=hparams.seed)
    gen_dm = None if only_classify else LatentPredDataModule(vqvae, splits, hparams.batch_size,
                                                             task="autoregressive_ids", seed=hparams.seed,
                                                             tokenized=cls_dm.tokenize())
    return vqvae.num_embeddings, vqvae.patch_size, cls_dm, gen_dm


def classification_finetuning(model, classification_epoch, logger, class_task_data_module, no_early_stopping=False,
                              n_gpus=1):
    early_stop_callback = EarlyStopping(monitor="val/cl/f1_score", min_delta=0.001, patience=5, verbose=False,
                                        mode="max")
    model.switch_to_classification()
    callbacks = [] if no_early_stopping else [early_stop_callback]
    trainer = Trainer(devices=n_gpus, num_nodes=1, max_epochs=classification_epoch, logger=logger,
                      callbacks=callbacks, gradient_clip_val=0.8, accumulate_grad_batches=5)
    trainer.fit(model, class_task_data_module)
    trainer = Trainer(devices=1, num_nodes=1, logger=logger, callbacks=callbacks)
    return trainer.test(model, class_task_data_module)


def main(hparams):
    if hparams.use_wandb or hparams.use_wandb_for_logging or hparams.use_mlflow:
        raise SystemExit("W&B / MLflow are not available in this build (no network); use the CSV logger")
    if hparams.model_wandb_transformer and not os.path.exists(hparams.model_wandb_transformer):
        raise SystemExit("--model-wandb-transformer must be a local checkpoint path in this build")
    set_operand_dtype(hparams.precision)
    # DDP only with --use-all-gpus (train_transformer_mtasks.py:149-153: otherwise Trainer(devices=1))
    rank, world, dev = init_distributed(enable=bool(hparams.use_all_gpus))
    logger = CSVLogger("logs", name="vq-vae-transformer")
    logger.log_hyperparams(vars(hparams))
    num_embeddings, patch_size, cls_dm, gen_dm = load_dataset(hparams, dev, only_classify=hparams.classification_only)
    seq_len = (hparams.n_cycles * (400 // patch_size)) + 1
    num_classes = num_embeddings + 2
    n_gpus = world if hparams.use_all_gpus else 1
    log.info(f"{n_gpus=}")
    log.info(f"{seq_len=} - {num_classes=} - {num_embeddings=} - {patch_size=}")
    torch.manual_seed(hparams.seed)
    if hparams.classification_only:
        if hparams.model_wandb_transformer:
            model = MyTransformerDecoder.load_from_checkpoint(hparams.model_wandb_transformer)
        else:
            model = MyTransformerDecoder(d_model=hparams.d_model, seq_len=seq_len, n_classes=num_classes,
                                         n_head=hparams.n_heads, n_blocks=hparams.n_blocks,
                                         class_h_bias=bool(hparams.use_class_head_bias),
                                         class_h_dropout=bool(hparams.use_class_head_dropout))
        model = model.to(dev)
        res = classification_finetuning(model, hparams.class_epoch, logger, cls_dm,
                                        no_early_stopping=hparams.no_early_stopping, n_gpus=n_gpus)
    else:
        model = MyTransformerDecoder(d_model=hparams.d_model, seq_len=seq_len, n_classes=num_classes,
                                     n_head=hparams.n_heads, n_blocks=hparams.n_blocks).to(dev)
        for epoch in range(hparams.epoch_iter):
            log.info("Generating stage")
            trainer = get_new_trainer(epochs_steps=hparams.gen_epochs, logger=logger, n_gpus=n_gpus)
            model.switch_to_generate()
            trainer.fit(model, gen_dm)
            if epoch == hparams.epoch_iter - 1:
                classification_finetuning(model, hparams.finetune_epochs, logger, cls_dm,
                                          no_early_stopping=hparams.no_early_stopping, n_gpus=n_gpus)
            else:
                trainer = get_new_trainer(epochs_steps=hparams.class_epoch, logger=logger, n_gpus=n_gpus)
                log.info("Classification stage")
                model.switch_to_classification()
                trainer.fit(model, cls_dm)
        trainer = get_new_trainer(epochs_steps=1, logger=logger, n_gpus=1)
        model.switch_to_classification()
        res = trainer.test(model, cls_dm)
        model.switch_to_generate()
        res += trainer.test(model, gen_dm)
    if rank == 0:
        print("test:", res)
        print("Done")
    shutdown()
    return res


def parser():
    p = argparse.ArgumentParser(description='Train-Latent-Transformer')
    p.add_argument('--epoch_iter', type=int, default=3)
    p.add_argument('--batch-size', type=int, help='Batch size', default=16)
    p.add_argument('--n-cycles', type=int, help='Number of cycles', default=20)
    p.add_argument('--d-model', type=int, default=512)
    p.add_argument('--n-heads', type=int, help='Number of heads', default=8)
    p.add_argument('--n-blocks', type=int, help='Number of transformer blocks', default=6)
    p.add_argument('--use-class-head-bias', action=argparse.BooleanOptionalAction)
    p.add_argument('--use-class-head-dropout', action=argparse.BooleanOptionalAction)
    p.add_argument('--use-wandb', action=argparse.BooleanOptionalAction)
    p.add_argument('--use-wandb-for-logging', action=argparse.BooleanOptionalAction)
    p.add_argument('--use-mlflow', action=argparse.BooleanOptionalAction)
    p.add_argument('--mlflow-url', type=str, default='')
    p.add_argument('--logging-entity', type=str)
    p.add_argument('--logging-project', type=str, default="asimow-vq-vae-transformer")
    p.add_argument('--vqvae-model', type=str, default="model_checkpoints/VQ-VAE-Patch/vq_vae_patch_best_01.ckpt")
    p.add_argument('--classification-only', action=argparse.BooleanOptionalAction)
    p.add_argument('--no-early-stopping', action=argparse.BooleanOptionalAction)
    p.add_argument('--class-epoch', type=int, help='Number of epochs for classification', default=2)
    p.add_argument('--finetune-epochs', type=int, help='Number of epochs for classification', default=10)
    p.add_argument('--model-wandb-transformer', type=str, default="")
    p.add_argument('--use-all-gpus', action=argparse.BooleanOptionalAction)
    # this build: generation epochs per stage (reference: fixed 10), synthetic data sizes, real-data .npz
    p.add_argument('--gen-epochs', type=int, default=10)
    p.add_argument('--n-train', type=int, default=1024)
    p.add_argument('--n-val', type=int, default=128)
    p.add_argument('--n-test', type=int, default=128)
    p.add_argument('--data-npz', type=str, default="")
    p.add_argument('--seed', type=int, default=0)
    p.add_argument('--precision', choices=["fp32", "bf16"], default="fp32",
                   help="MFMA operand dtype (bf16: opt-in, fp32 accumulation and master weights)")
    return p


if __name__ == '__main__':
    args = parser().parse_args()
    log.basicConfig(level=log.INFO, format='%(asctime)s - %(levelname)s - %(message)s')
    torch.set_float32_matmul_precision('medium')
    main(args)

"""Drop-in for the reference's AIR training entry point
(training_air_original.py): same command line (-r -k -gpu -data -o -t -dn -dl
-ds -ap), same dataset paths, results folder, model configuration and log
lines, running the AIR train step on MI355X through mog_air.AIRModel.

    python training_air_original.py -dn 13 -ds 20k [--iterations N] [--precision bf16]

Model configuration: training_air_original.py:158-211 (max_steps 6, LSTM 256,
VAE 784-512-256-50, scale prior -1 / 0.05, lr 1e-4, clip 1.0, z_pres prior
log-odds annealed from 1e4 by 0.1 per 3000 iterations in log space).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mog-asr_amd"))

MAX_STEPS = 6
NUM_IMAGES_TO_SAVE = 60


def main(argv=None):
    from mog_air import trainer
    parser = argparse.ArgumentParser()
    trainer.add_common_args(parser, reader_threads=4)
    parser.add_argument("-ap", "--add_prior", type=str, default="")
    args = parser.parse_args(argv)
    args.add_prior = args.add_prior.lower() in ["true", "t", "1"]
    trainer.select_gpu(args.gpu)  # before the HIP runtime starts

    import numpy as np
    np.random.seed(1234)
    from mog_air.air_model import AIRModel

    train_file, test_file, canvas, name, digits = trainer.dataset_files(args, "training_air_original.py")
    ctx = trainer.distributed_setup(args)  # one process per GPU under torch.distributed.run
    folder = trainer.results_folder(args, "training_air_original.py", name, main=ctx.main)
    log = trainer.build_logger(folder, args, main=ctx.main)
    if ctx.main:
        trainer.copy_sources(folder, [ROOT, os.path.join(ROOT, "mog-asr_amd", "mog_air")])

    log.info("Creating input pipeline...")
    if not ctx.main:
        ctx.barrier()  # rank 0 writes synthetic data first when asked to
    tr_x, tr_k, test = trainer.load_data(args, train_file, test_file, digits, log)
    if ctx.main:
        ctx.barrier()

    models = []
    for i in range(2):
        print("Creating {0} model...".format("training" if i == 0 else "testing"))
        models.append(AIRModel(
            None, None, max_steps=MAX_STEPS, max_digits=MAX_STEPS, rnn_units=256,
            canvas_size=canvas, windows_size=28, vae_latent_dimensions=50,
            vae_recognition_units=(512, 256), vae_generative_units=(256, 512),
            scale_prior_mean=-1.0, scale_prior_variance=0.05, shift_prior_mean=0.0,
            shift_prior_variance=1.0, vae_prior_mean=0.0, vae_prior_variance=1.0,
            vae_likelihood_std=0.3, scale_hidden_units=64, shift_hidden_units=64,
            z_pres_hidden_units=64, z_pres_prior_log_odds=-0.01, z_pres_temperature=1.0,
            stopping_threshold=0.99, learning_rate=1e-4, gradient_clipping_norm=1.0,
            cnn=False, cnn_filters=8, num_summary_images=NUM_IMAGES_TO_SAVE,
            train=(i == 0), reuse=(i == 1), scope="air",
            annealing_schedules={"z_pres_prior_log_odds": {
                "init": 10000.0, "min": 0.000000001, "factor": 0.1, "iters": 3000,
                "staircase": False, "log": True}},
            num_prior=digits if args.add_prior else None,
            device=args.device, seed=1235, precision=args.precision,
            noise_seed=1235 + ctx.rank,  # independent Monte-Carlo noise per rank
            grad_world=ctx.world if i == 0 else 1))
    train_model, test_model = models
    trainer.attach_data_parallel(train_model, ctx)
    log.info("Initializing variables...")
    return trainer.train_loop(args, train_model, test_model, tr_x, tr_k, test, canvas, log,
                              os.path.join(folder, "models"), ctx=ctx)


if __name__ == "__main__":
    main()

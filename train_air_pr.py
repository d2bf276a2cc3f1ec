"""Drop-in for the reference's AIR-ASR training entry point (train_air_pr.py):
same command line (-r -k -gpu -data -gl -gn -gne -gm -gb -gs -ga -zt -o -t -dn
-dl -ds), dataset paths, results folder, model configuration and log lines,
running the ASR model (mog_air.asr_model.AIRModel, the reference's
air/air_number_bbox_location.py) on MI355X.

    python train_air_pr.py -dn 13 -ds 20k -gm 100 -gne 10 [--iterations N]

Model configuration: train_air_pr.py:160-213 (max_steps 6, LSTM 256, VAE
784-512-256-50 with likelihood std 0, fixed scale prior, threshold 0.9,
temperature -zt, lr 1e-4, clip 1.0, number / bbox / size / area
regularisers from the -g* flags, fix_steps when -dn names one count).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mog-asr_amd"))

MAX_STEPS = 6
NUM_IMAGES_TO_SAVE = 64


def main(argv=None):
    from mog_air import trainer
    parser = argparse.ArgumentParser()
    trainer.add_common_args(parser, reader_threads=1)
    parser.add_argument("-gl", "-gamma_location", "--gamma_location", type=float, default=0.0)
    parser.add_argument("-gn", "-gamma_number", "--gamma_number", type=float, default=0.0)
    parser.add_argument("-gne", "-gamma_number_element", "--gamma_number_element", type=float,
                        default=0.0)
    parser.add_argument("-gm", "-gamma_margin", "--gamma_margin", type=float, default=0.0)
    parser.add_argument("-gb", "-gamma_bbox", "--gamma_bbox", type=float, default=0.0)
    parser.add_argument("-gs", "-gamma_size", "--gamma_size", type=float, default=0.0)
    parser.add_argument("-ga", "-gamma_area", "--gamma_area", type=float, default=0.0)
    parser.add_argument("-zt", "-z_pres_tempture", "--z_pres_tempture", type=float, default=0.1)
    args = parser.parse_args(argv)
    trainer.select_gpu(args.gpu)

    import numpy as np
    np.random.seed(1234)
    from mog_air.asr_model import AIRModel

    train_file, test_file, canvas, name, digits = trainer.dataset_files(args, "train_air_pr.py")
    if args.data.lower() == "mnist":
        size_min, size_max = (11, 15) if "bbox" in args.dig_surfix else (17, 23)
    else:
        size_min, size_max = (12, 15) if "bbox" in args.dig_surfix else (20, 25)
    print(size_min, size_max)
    ctx = trainer.distributed_setup(args)  # one process per GPU under torch.distributed.run
    folder = trainer.results_folder(args, "train_air_pr.py", name, main=ctx.main)
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
            fix_scale_distribution=True, vae_prior_mean=0.0, vae_prior_variance=1.0,
            vae_likelihood_std=0.0, scale_hidden_units=64, shift_hidden_units=64,
            z_pres_hidden_units=64, z_pres_prior_log_odds=-0.01,
            z_pres_temperature=args.z_pres_tempture, stopping_threshold=0.9,
            learning_rate=1e-4, gradient_clipping_norm=1.0, cnn=False, cnn_filters=8,
            num_summary_images=NUM_IMAGES_TO_SAVE, train=(i == 0), reuse=(i == 1), scope="air",
            constrains_x_y=None, constrains_num=digits, constrains_num_gamma=args.gamma_number,
            constrains_margin_gamma=args.gamma_margin,
            constrains_num_element_gamma=args.gamma_number_element,
            constrains_bbox_gamma=args.gamma_bbox, constrains_sharesize_gamma=args.gamma_size,
            constrains_area_gamma=args.gamma_area, constrains_area_minmax=[size_min, size_max],
            fix_steps=digits[0] if len(digits) == 1 else None, annealing_schedules={},
            device=args.device, seed=1235, precision=args.precision,
            noise_seed=1235 + ctx.rank,  # independent Monte-Carlo noise per rank
            grad_world=ctx.world if i == 0 else 1))
    train_model, test_model = models
    trainer.attach_data_parallel(train_model, ctx)
    log.info("Initializing variables...")
    return trainer.train_loop_asr(args, train_model, test_model, tr_x, tr_k, test, canvas, log,
                                  os.path.join(folder, "models"), ctx=ctx)


if __name__ == "__main__":
    main()

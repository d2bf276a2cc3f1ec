"""Training driver behind the kept entry points (training_air_original.py,
train_air_pr.py): results-folder handling, logging, the input pipeline, the
train / test model pair sharing one variable scope, the iteration loop with
the reference's logging / testing / checkpoint cadence, and the end-of-data
(OutOfRangeError) epilogue — training_air_original.py:18-503 and
train_air_pr.py:18-400 restated around ``AIRModel.step`` / ``infer``.

Image grids (training_air_original.py:368-411, :445-490): every
IMAGE_SAVE_ITERATION iterations and at the end, the test model's
reconstruction / misclassified / generation grids are written as PNG files
under summary/ (``mog_air.visualize``).  TensorBoard event files are out of
scope.
"""
from __future__ import annotations

import glob
import logging
import operator
import os
import shutil
import time
from typing import Optional

import numpy as np

from . import records
from .evaluation import evaluation

EPOCHS = 300
BATCH_SIZE = 64
LOG_EACH_ITERATION = 20
TEST_EACH_ITERATION = 200
IMAGE_SAVE_ITERATION = 500  # training_air_original.py:31
NUM_IMAGES_TO_SAVE = 60     # :43
SAVE_PARAMS_EACH_ITERATIONS = 10000


def add_common_args(parser, reader_threads: int):
    """The CLI flags shared by both entry points (training_air_original.py:49-60,
    train_air_pr.py:40-61) plus this framework's options (not in the
    reference): --iterations, --precision, --test-batch, --synth-per-count,
    --write-synthetic, --device."""
    parser.add_argument("-r", "--results-folder", default="Not Valid")
    parser.add_argument("-k", "-key", "--key", default="")
    parser.add_argument("-gpu", "--gpu", default="-1")
    parser.add_argument("-data", "--data", default="mnist")
    parser.add_argument("-o", "--overwrite-results", type=int, choices=[0, 1], default=0)
    parser.add_argument("-t", "--reader-threads", type=int, default=reader_threads)
    parser.add_argument("-dn", "--dig_num", type=str, default="02")
    parser.add_argument("-dl", "--dig_location", type=str, default="")
    parser.add_argument("-ds", "--dig_surfix", type=str, default="")
    parser.add_argument("--iterations", type=int, default=0,
                        help="stop after this many train iterations (0: run all epochs)")
    parser.add_argument("--precision", choices=["fp32", "bf16"], default="fp32")
    parser.add_argument("--test-batch", type=int, default=0,
                        help="test-set images per test-model launch (0: whole set)")
    parser.add_argument("--synth-per-count", type=int, default=2000,
                        help="images per object count when the dataset files are absent")
    parser.add_argument("--write-synthetic", type=int, choices=[0, 1], default=0)
    parser.add_argument("--device", default="cuda:0")
    parser.add_argument("--no-images", action="store_true",
                        help="skip the PNG grids (training_air_original.py:368-411)")


def select_gpu(gpu: str) -> None:
    """-gpu N (training_air_original.py:64-65): must run before the HIP runtime
    starts; HIP_VISIBLE_DEVICES is the ROCm spelling of CUDA_VISIBLE_DEVICES.
    Under torch.distributed.run (WORLD_SIZE > 1) each rank takes the GPU of
    its LOCAL_RANK instead (distributed_setup)."""
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return
    if 0 <= int(gpu) <= 7:
        os.environ["HIP_VISIBLE_DEVICES"] = str(gpu)


class Dist:
    """Data-parallel context of one trainer process: rank,
    world, the contiguous shard of each global batch this rank trains on."""

    def __init__(self, rank: int = 0, world: int = 1):
        self.rank, self.world = rank, world

    @property
    def main(self) -> bool:
        return self.rank == 0

    def shard(self, x, k):
        """This rank's contiguous part of a global batch."""
        if self.world == 1:
            return x, k
        from .parallel import shard
        lo, hi = shard(len(k), self.rank, self.world)
        return x[lo:hi], k[lo:hi]

    def mean(self, values, device, weight: float = 1.0):
        """Weighted mean over ranks of a few host scalars (one small
        all-reduce): each rank's values are per-image means over its shard, so
        weighting by the shard size (``weight``) gives the global batch mean
        even when the shards differ in size (a global batch that does not
        divide by the world size)."""
        if self.world == 1:
            return list(values)
        import torch
        import torch.distributed as dist
        t = torch.tensor([float(v) * weight for v in values] + [float(weight)],
                         dtype=torch.float64, device=device)
        dist.all_reduce(t)
        return (t[:-1] / t[-1]).tolist()

    def barrier(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.barrier()


def distributed_setup(args) -> Dist:
    """One process per GPU under torch.distributed.run: RCCL ("nccl") process
    group, device = cuda:LOCAL_RANK (written into args.device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1:
        return Dist()
    import torch
    import torch.distributed as dist
    local = int(os.environ.get("LOCAL_RANK", "0"))
    args.device = "cuda:%d" % local
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device(args.device))
    return Dist(dist.get_rank(), world)


def attach_data_parallel(train_model, ctx: Dist) -> None:
    if ctx.world > 1:
        from .parallel import attach
        attach(train_model)


def dataset_files(args, entry: str):
    """(train file, test file, canvas size, common name), as the entry points
    derive them from -data/-dn/-dl/-ds (training_air_original.py:67-91)."""
    digits = [int(c) for c in args.dig_num]
    if args.dig_location not in ["", "right_half"]:
        raise ValueError("not valid location of digit: " + args.dig_location)
    name = args.dig_location + args.dig_surfix + "".join(str(d) for d in digits)
    if args.data.lower() == "mnist":
        folder, canvas = "./data/multi_mnist_data/", 50
    else:
        folder, canvas = "./data/multi_dsprites/", 64
    return (os.path.join(folder, f"common{name}.tfrecords"),
            os.path.join(folder, f"test{name}.tfrecords"), canvas, name, digits)


def results_folder(args, entry: str, name: str, main: bool = True) -> str:
    """training_air_original.py:93-115: default name, -k suffix, -o overwrite
    or the next free _N suffix; creates models/, summary/, source/ (rank 0
    only when data parallel — the other ranks write nothing)."""
    if args.results_folder == "Not Valid":
        args.results_folder = "./results/{time}-({file}_{data})_(train.{train}_test.{test})".format(
            file=entry, train=name.replace("_", "."), test=name.replace("_", "."),
            time=time.strftime("%Y-%m-%d-%H-%M"), data=args.data)
    args.results_folder += "_({})".format(args.key)
    if not main:
        return args.results_folder
    if os.path.exists(args.results_folder):
        if args.overwrite_results:
            shutil.rmtree(args.results_folder, ignore_errors=True)
        else:
            base, i = args.results_folder, 0
            args.results_folder = f"{base}_{i}"
            while os.path.exists(args.results_folder):
                i += 1
                args.results_folder = f"{base}_{i}"
    for sub in ("", "models", "summary", "source"):
        os.makedirs(os.path.join(args.results_folder, sub), exist_ok=True)
    return args.results_folder


def build_logger(folder: str, args, main: bool = True) -> logging.Logger:
    """utils/checkpoints.py:31-63: console + results-folder log file, then the
    sorted configurable parameters between '#' rules (rank 0 only when data
    parallel; the other ranks log nothing)."""
    fmt = "%(asctime)s;%(levelname)s|%(message)s"
    log = logging.getLogger("mog_air")
    log.setLevel(logging.INFO)
    log.propagate = False
    for h in list(log.handlers):
        log.removeHandler(h)
    if not main:
        log.addHandler(logging.NullHandler())
        return log
    sh = logging.StreamHandler()
    sh.setFormatter(logging.Formatter(fmt, "%H-%M-%S"))
    log.addHandler(sh)
    fh = logging.FileHandler(os.path.join(folder, "logfile{}.log".format(time.strftime("%m-%d"))))
    fh.setFormatter(logging.Formatter(fmt, "%H:%M:%S"))
    log.addHandler(fh)
    log.info("#" * 120)
    log.info("----------Configurable Parameters In this Model----------")
    for k, v in sorted(vars(args).items(), key=operator.itemgetter(0)):
        log.info("# " + ("%20s" % k) + ":\t" + str(v))
    log.info("#" * 120)
    return log


def copy_sources(folder: str, roots) -> None:
    """training_air_original.py:128-135: snapshot of the *.py sources."""
    for src in roots:
        dst = os.path.join(folder, "source", os.path.basename(os.path.normpath(src))
                           if src not in (".", "./") else "")
        os.makedirs(dst, exist_ok=True)
        for f in glob.glob(os.path.join(src, "*.py")):
            shutil.copy(f, dst)


def load_data(args, train_file, test_file, digits, log):
    """Train arrays + test tuple (read_test_data).  When the files are absent
    (the reference builds them from MNIST, which needs the network), an
    offline synthetic dataset of the same layout is generated (datasets.py)
    and optionally written to the expected paths."""
    if os.path.exists(train_file) and os.path.exists(test_file):
        log.info("Reading %s and %s", train_file, test_file)
        tr_x, tr_k = records.load_images(train_file)
        test = records.read_test_data(test_file, shift_zero_digits_images=True)
        return tr_x, tr_k, test
    from . import datasets
    log.warning("dataset files %s / %s not found: synthesizing an offline stand-in "
                "(%d images per object count)", train_file, test_file, args.synth_per_count)
    kind = "mnist" if args.data.lower() == "mnist" else "dsprites"
    sets = datasets.synthesize(kind, digits, args.synth_per_count,
                               test_set_size=min(1000, args.synth_per_count * len(digits) // 5),
                               seed=0, bbox="bbox" in args.dig_surfix)
    if args.write_synthetic:
        for path, split in ((train_file, "train"), (test_file, "test")):
            os.makedirs(os.path.dirname(path), exist_ok=True)
            s = sets[split]
            records.write_to_records(path[:-len(".tfrecords")], s["images"], s["indices"],
                                     s["positions"], s["boxes"], s["labels"], s["digits"])
        return load_data(args, train_file, test_file, digits, log)
    tr = sets["train"]
    tr_x = np.stack([im.ravel() for im in tr["images"]]).astype(np.float32)
    tr_k = np.asarray(tr["digits"], np.int32)
    te = sets["test"]
    test = (np.stack([im.ravel() for im in te["images"]]).astype(np.float32),
            np.asarray(te["digits"], np.int32), [np.asarray(v, np.int32) for v in te["indices"]],
            [np.asarray(v, np.int32) for v in te["positions"]],
            [np.asarray(v, np.int32) for v in te["boxes"]],
            [np.asarray(v, np.int32) for v in te["labels"]])
    return tr_x, tr_k, test


class Saver:
    """tf.train.Saver(max_to_keep=3) stand-in: <folder>/<prefix>-<step>.npz
    holding every variable under its TF name."""

    def __init__(self, folder: str, prefix: str, max_to_keep: int = 3):
        self.folder, self.prefix, self.keep = folder, prefix, max_to_keep
        self.saved = []

    def save(self, params, step: int) -> str:
        path = os.path.join(self.folder, f"{self.prefix}-{step}.npz")
        np.savez(path, **{k.replace("/", "__"): v for k, v in params.state_dict().items()})
        self.saved.append(path)
        while len(self.saved) > self.keep:
            old = self.saved.pop(0)
            if os.path.exists(old):
                os.remove(old)
        return path


def run_test(test_model, test, canvas: int, batch: int):
    """Test-model fetches over the whole test set: (loss, accuracy, mse,
    rec_scales, rec_shifts, rec_num_digits), batched when `batch` > 0 and
    combined as the batch means the reference computes in one run."""
    images, digits = test[0], test[1]
    n = len(digits)
    step = batch if batch > 0 else n
    loss = acc = mse = 0.0
    scales, shifts, nums = [], [], []
    T = test_model.max_steps
    for s in range(0, n, step):
        x, k = images[s:s + step], digits[s:s + step]
        test_model.infer(x, k)
        w = len(k) / n
        loss += test_model.loss * w
        acc += test_model.accuracy * w
        mse += test_model.mse_loss * w
        sc = np.zeros((len(k), T, 1), np.float32)
        sh = np.zeros((len(k), T, 2), np.float32)
        rs, rh = test_model.rec_scales.cpu().numpy(), test_model.rec_shifts.cpu().numpy()
        sc[:, :rs.shape[1]] = rs
        sh[:, :rh.shape[1]] = rh
        scales.append(sc)
        shifts.append(sh)
        nums.append(test_model.rec_num_digits.cpu().numpy())
    return loss, acc, mse, np.concatenate(scales), np.concatenate(shifts), np.concatenate(nums)


def train_loop(args, train_model, test_model, tr_x, tr_k, test, canvas, log, models_folder,
               extra_log=None, ctx: Optional[Dist] = None):
    """The iteration loop of training_air_original.py:226-503 (logging every
    20, testing every 200, parameters every 10,000 iterations; the final
    test when the input runs out)."""
    ctx = ctx or Dist()
    batcher = records.ShuffleBatcher(tr_x, tr_k, BATCH_SIZE, EPOCHS,
                                     min_after_dequeue=min(10000, len(tr_k)))
    saver = Saver(models_folder, "air-model")
    min_loss, update_flag = 9999999.0, False
    best = [0.0, 0.0, 0.0, 0.0]
    hist = []
    step = 0

    def test_and_log(tag):
        nonlocal update_flag
        if not ctx.main:
            ctx.barrier()
            return 0.0, 0.0, 0.0, 0.0
        tl, ta, tm, sc, sh, nd = run_test(test_model, test, canvas, args.test_batch)
        ctx.barrier()
        log.info("iteration {}\ttest loss {:.3f}\ttest accuracy {:.2f}, test mse {:.3f}".format(
            tag, tl, ta, tm))
        p, r, gt_iou, det_iou, g_iou = evaluation(test[3], test[4], sh, sc, nd, csize=canvas)
        # integer steps are padded to 6 as training_air_original.py:357 does
        # ('final' is printed as is)
        step_tag = "{:6d}".format(tag) if isinstance(tag, int) else tag
        log.info("test:{}\tprecision:{}\trecall:{}\tgtIoU:{:.4f}\tdetectionIoU:{:.4f}"
                 "\tglobaliou:{:.4f}".format(step_tag, p, r, gt_iou, det_iou, g_iou))
        return tl, ta, tm, g_iou

    summary_folder = os.path.join(os.path.dirname(os.path.normpath(models_folder)), "summary")
    digits = [int(c) for c in getattr(args, "dig_num", "")]
    vis_n = args.test_batch if getattr(args, "test_batch", 0) > 0 else len(test[1])

    def save_images(tag, generations=True, gen_tag=None):
        if not ctx.main or getattr(args, "no_images", False):
            return
        from .visualize import save_visualizations
        save_visualizations(test_model, test[0][:vis_n], test[1][:vis_n], summary_folder, tag,
                            digits=digits, num=NUM_IMAGES_TO_SAVE, generations=generations,
                            gen_tag=gen_tag)

    log.info("Training...\n")
    try:
        while True:
            if step % SAVE_PARAMS_EACH_ITERATIONS == 0 and ctx.main:
                saver.save(train_model.params, step)
            xg, kg = batcher.next_batch()
            x, k = ctx.shard(xg, kg)
            loss, acc, mse, step = train_model.step(x, k, global_batch=len(kg))
            if extra_log is not None:
                extra_log(train_model, step)
            hist.append([loss, acc, mse])
            if step % LOG_EACH_ITERATION == 0:
                l0, l1, l2 = ctx.mean(np.mean(hist[-LOG_EACH_ITERATION:], axis=0), args.device,
                                      weight=len(k))
                log.info("iteration {}\ttrain loss {:.3f}\ttrain accuracy {:.2f}, "
                         "train mse {:.3f}".format(step, l0, l1, l2))
                if l0 < min_loss:
                    update_flag, min_loss = True, l0
            if step % TEST_EACH_ITERATION == 0:
                tl, ta, tm, g_iou = test_and_log(step)
                if update_flag:
                    update_flag = False
                    best = [tl, ta, tm, g_iou]
                log.info("Current Best: elbo:{}\taccu:{}\tmse:{}\tiou:{}".format(*best))
            if step % IMAGE_SAVE_ITERATION == 0:
                save_images(step)
            if args.iterations and step >= args.iterations:
                raise StopIteration
    except StopIteration:
        test_and_log("final")
        # the final reconstruction / misclassified grids are tagged 'final',
        # the final generation grids with the step (training_air_original.py:478-483)
        save_images("final", gen_tag=step)
        log.info("Final Best: elbo:{}\taccu:{}\tmse:{}\tiou:{}".format(*best))
        log.info("\ntraining has ended\n")
    return step


TESET_EACH_ITERATION = 200  # (sic) train_air_pr.py:31


def train_loop_asr(args, train_model, test_model, tr_x, tr_k, test, canvas, log, models_folder,
                   ctx: Optional[Dist] = None):
    """The iteration loop of train_air_pr.py:284-400: every step fetches the
    model's log variables; every 20 iterations their means are logged, every
    200 the test model runs on the test set (log variables + detection
    metrics); parameters are saved every 10,000 iterations; the final test
    when the input runs out.  Data parallel as train_loop."""
    ctx = ctx or Dist()
    batcher = records.ShuffleBatcher(tr_x, tr_k, BATCH_SIZE, EPOCHS,
                                     min_after_dequeue=min(10000, len(tr_k)))
    saver = Saver(models_folder, "air-model")
    min_loss, update_flag = 9999999.0, False
    best = [0.0, 0.0, 0.0, 0.0]
    logged = {}
    step = 0

    def test_and_log(tag):
        nonlocal update_flag
        if not ctx.main:
            ctx.barrier()
            return
        tl, ta, tm, sc, sh, nd = run_test(test_model, test, canvas, args.test_batch)
        ctx.barrier()
        p, r, gt_iou, det_iou, g_iou = evaluation(test[3], test[4], sh, sc, nd, csize=canvas)
        log.info("test:{:6d}\tprecision:{}\trecall:{}\tgtIoU:{:.4f}\tdetectionIoU:{:.4f}"
                 "\tglobal_iou:{:.4f}".format(tag, p, r, gt_iou, det_iou, g_iou))
        lv = test_model.log_variables
        if update_flag:
            update_flag = False
            best[:] = [lv["elbo"], lv["accu"], lv["mse"], g_iou]
        log.info("test:{:6d}\t".format(tag) +
                 "".join("{}:{:.4f}\t".format(n, v) for n, v in lv.items()))
        log.info("Current Best: elbo:{}\taccu:{}\tmse:{}\tiou:{}".format(*best))

    summary_folder = os.path.join(os.path.dirname(os.path.normpath(models_folder)), "summary")
    vis_n = args.test_batch if getattr(args, "test_batch", 0) > 0 else len(test[1])

    def save_images(tag):
        # train_air_pr.py:362-389 (the ASR generation grids need the
        # generative LSTM prior, not part of this build)
        if not ctx.main or getattr(args, "no_images", False):
            return
        from .visualize import save_visualizations
        save_visualizations(test_model, test[0][:vis_n], test[1][:vis_n], summary_folder, tag,
                            num=NUM_IMAGES_TO_SAVE, generations=False)

    log.info("Training...\n")
    try:
        while True:
            if step % SAVE_PARAMS_EACH_ITERATIONS == 0 and ctx.main:
                saver.save(train_model.params, step)
            xg, kg = batcher.next_batch()
            x, k = ctx.shard(xg, kg)
            _, _, _, step = train_model.step(x, k, global_batch=len(kg))
            for n, v in train_model.log_variables.items():
                logged.setdefault(n, []).append(v)
            if step % LOG_EACH_ITERATION == 0:
                line = "step:{:6d}\t".format(step)
                # the global batch's means (shard-size weighted over ranks)
                means = ctx.mean([np.mean(v) for v in logged.values()], args.device,
                                 weight=len(k))
                for n, v in zip(logged, means):
                    if n == "TotLoss" and v < min_loss:
                        min_loss, update_flag = float(v), True
                    line += "{}:{:.4f}\t".format(n, v)
                log.info(line)
                logged = {}
            if step % TESET_EACH_ITERATION == 0:
                test_and_log(step)
            if step % IMAGE_SAVE_ITERATION == 0:
                save_images(step)
            if args.iterations and step >= args.iterations:
                raise StopIteration
    except StopIteration:
        test_and_log(step)  # the reference logs the step here too (train_air_pr.py:426-430)
        save_images("final")
        log.info("Final Best: elbo:{}\taccu:{}\tmse:{}\tiou:{}".format(*best))
        log.info("\ntraining has ended\n")
    return step

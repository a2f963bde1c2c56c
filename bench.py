"""bench.py -- frames/sec of one training step (fwd + bwd + update) of the
BASELINE stack Conv(40x11x3, 8x1, 128) -> Maxpool(1x1x4) -> FC(11616 -> 1024)
on MI355X through libkcnn.so, plus the dominant hot-path kernel's roofline
fraction (HIP events over the timed region) and the CPU oracle timed on the
host beside it.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--frames-per-gpu B]

N > 1 runs under torch.distributed.run, one process per GPU (started by
bench.py itself as a child `python -m torch.distributed.run` when no launcher
set WORLD_SIZE, so `python bench.py --gpus N` runs N ranks): the minibatch is
row-sharded (weak scaling, B frames per GPU), gradients are computed per
component and all-reduced over RCCL (sum, fp32) while the lower layers
backpropagate, then every replica applies the same update with
lr / (B * N).  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kaldi-cnn_amd"))

# BASELINE.json configs[1] (c2).
H, W, C, KH, KW, G, PC, FC_OUT = 40, 11, 3, 8, 1, 128, 4, 1024
OH, OW = H - KH + 1, W - KW + 1
P = OH * OW
POOL_OUT = P * G // PC
PEAK_HBM_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
PEAK_FP32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md: fp32 matrix (dense)
PEAK_BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: bf16 matrix (dense, spec)
PEAK_F16_MFMA_TFLOPS = 2500.0   # MI355X_MICROARCH.md: f16 matrix (dense, spec; = bf16)
# fp32-equivalent ceiling of each engine the kernels run fp32 products on:
# the dense peak of its matrix type over its products per fp32 product
ENGINE_PEAK_TFLOPS = {"fp32": PEAK_FP32_MFMA_TFLOPS, "bf16x6": PEAK_BF16_MFMA_TFLOPS / 6,
                      "f16x3": PEAK_F16_MFMA_TFLOPS / 3}

# Algorithmic work per frame (SURVEY 8d / BASELINE.md 3).
CONV_FLOP_PER_PASS = 2 * P * G * KH * KW * C          # 2,230,272
CONV_BYTES_PER_PASS = 4 * (H * W * C + P * G)         # 191,136
CONV_BWD_BYTES = 4 * (2 * H * W * C + P * G)          # 196,416: X, dY in; dX out
CONV_BWD_FLOP = 2 * CONV_FLOP_PER_PASS                # dgrad + wgrad
CONV_BIAS_GRAD_FLOP = 2 * P * G                        # the bias gradient, reported apart
POOL_FWD_BYTES = 4 * (P * G + POOL_OUT)               # 232,320
POOL_BWD_BYTES = 4 * (2 * P * G + 2 * POOL_OUT)       # 464,640
# Conv -> Maxpool run fused by the kcnn_nnet runtime (kcnn_set_fusion):
# forward reads X, writes the pooled output and a 1-byte routing mask (and Y
# only with --store-conv-out: nothing in the step reads it); the pool
# backward reads the mask and dP and writes dY.
CONV_POOL_FWD_BYTES = 4 * (H * W * C + POOL_OUT) + POOL_OUT          # 63,360
CONV_POOL_FWD_Y_BYTES = CONV_POOL_FWD_BYTES + 4 * P * G             # 249,216
# Maxpool backward folded into the conv backward (fusion mode 1): reads X,
# dP and the mask, writes dX; dY is built slab by slab in LDS
CONV_BWD_POOLED_BYTES = 4 * (2 * H * W * C + POOL_OUT) + POOL_OUT    # 68,640
POOL_BWD_MASK_BYTES = POOL_OUT + 4 * (POOL_OUT + P * G)               # 243,936
FC_FLOP = 3 * 2 * POOL_OUT * FC_OUT                   # 71,368,704
DY_RING = 8   # synthetic output derivatives cycled over the steps (4 and their negations)


def stack_config():
    return "\n".join([
        f"ConvolutionComponent in-height={H} in-width={W} in-channel={C} "
        f"kernel-height={KH} kernel-width={KW} stride=1 group={G} out-height={OH} "
        f"out-width={OW} learning-rate=0.02 param-stddev=0.01 bias-stddev=0.5 "
        f"weight-decay=0.0002 momentum=0.9",
        f"MaxpoolComponent in-height={OH} in-width={OW} in-channel={G} "
        f"pool-height-dim=1 pool-width-dim=1 pool-channel-dim={PC}",
        f"FullyConnectedComponent input-dim={POOL_OUT} output-dim={FC_OUT} "
        f"learning-rate=0.02 param-stddev=0.01 bias-stddev=1 weight-decay=0.0002 "
        f"momentum=0.9",
    ])


# BASELINE configs[4] / SURVEY 8d c5: the deep stack, (H, W, C, kh, kw, G, pad)
# convolutions and (ph, pw, pc) pools, FC(1792 -> 1024).  A --config option;
# the default line stays c2 (the configuration BASELINE's metric is quoted on).
C5_LAYERS = [
    ("conv", (40, 11, 3, 8, 1, 256, 0)),
    ("pool", (3, 1, 4)),
    ("conv", (11, 11, 64, 4, 3, 256, 0)),
    ("conv", (8, 9, 256, 3, 3, 256, 1)),
    ("pool", (2, 1, 4)),
    ("conv", (4, 9, 64, 4, 3, 256, 0)),
]


def c5_config():
    lines, shape = [], None
    flop = 0
    for kind, a in C5_LAYERS:
        if kind == "conv":
            h, w, c, kh, kw, g, pad = a
            oh, ow = h + 2 * pad - kh + 1, w + 2 * pad - kw + 1
            lines.append(
                f"ConvolutionComponent in-height={h} in-width={w} in-channel={c} "
                f"in-pad-height={pad} in-pad-width={pad} kernel-height={kh} "
                f"kernel-width={kw} stride=1 group={g} out-height={oh} out-width={ow} "
                f"learning-rate=0.02 param-stddev=0.01 bias-stddev=0.5")
            flop += 2 * oh * ow * g * kh * kw * c
            shape = (oh, ow, g)
        else:
            ph, pw, pc = a
            oh, ow, g = shape
            lines.append(f"MaxpoolComponent in-height={oh} in-width={ow} in-channel={g} "
                         f"pool-height-dim={ph} pool-width-dim={pw} pool-channel-dim={pc}")
            shape = (oh // ph, ow // pw, g // pc)
    fin = shape[0] * shape[1] * shape[2]
    lines.append(f"FullyConnectedComponent input-dim={fin} output-dim={FC_OUT} "
                 f"learning-rate=0.02 param-stddev=0.01 bias-stddev=1")
    return "\n".join(lines), flop, fin


# The reference's own model, egs/exp/nnet/nnet.config, through its last
# FullyConnectedComponent: Splice(40, +-10) -> 6 x (Conv -> ReLU) with a
# 1x2x1 Maxpool -> FC 1024 -> 4096 -> 4096 -> 3454 with ReLUs.  The two
# DropoutComponents and the SoftmaxComponent are not part of this build (the
# output derivative is synthetic, as for c2/c5), and the last FC is
# initialised like the others (param-stddev 0.01, bias-stddev 1) instead of
# all-zero, so no layer trains on zeros.
NNET_CONFIG = """SpliceComponent input-dim=40 left-context=10 right-context=10 const-component-dim=0
ConvolutionComponent in-height=40 in-width=21 in-channel=1 kernel-height=40 kernel-width=4 stride=1 group=128 out-height=1 out-width=18 learning-rate=0.02 param-stddev=0.01 bias-stddev=0.5 weight-decay=0.0005 momentum=0.9
RectifiedLinearComponent dim=2304
ConvolutionComponent in-height=1 in-width=18 in-channel=128 kernel-height=1 kernel-width=3 stride=1 group=128 out-height=1 out-width=16 learning-rate=0.02 param-stddev=0.01 bias-stddev=0.5 weight-decay=0.0005 momentum=0.9
RectifiedLinearComponent dim=2048
ConvolutionComponent in-height=1 in-width=16 in-channel=128 kernel-height=1 kernel-width=3 stride=1 group=256 out-height=1 out-width=14 learning-rate=0.02 param-stddev=0.01 bias-stddev=0.5 weight-decay=0.0005 momentum=0.9
RectifiedLinearComponent dim=3584
ConvolutionComponent in-height=1 in-width=14 in-channel=256 kernel-height=1 kernel-width=3 stride=1 group=256 out-height=1 out-width=12 learning-rate=0.02 param-stddev=0.01 bias-stddev=0.5 weight-decay=0.0005 momentum=0.9
MaxpoolComponent in-height=1 in-width=12 in-channel=256 pool-height-dim=1 pool-width-dim=2 pool-channel-dim=1
RectifiedLinearComponent dim=1536
ConvolutionComponent in-height=1 in-width=6 in-channel=256 kernel-height=1 kernel-width=3 stride=1 group=512 out-height=1 out-width=4 learning-rate=0.02 param-stddev=0.01 bias-stddev=0.5 weight-decay=0.0005 momentum=0.9
RectifiedLinearComponent dim=2048
ConvolutionComponent in-height=1 in-width=4 in-channel=512 kernel-height=1 kernel-width=3 stride=1 group=512 out-height=1 out-width=2 learning-rate=0.02 param-stddev=0.01 bias-stddev=0.5 weight-decay=0.0005 momentum=0.9
RectifiedLinearComponent dim=1024
FullyConnectedComponent input-dim=1024 output-dim=4096 learning-rate=0.02 param-stddev=0.01 bias-stddev=1 weight-decay=0.0005 momentum=0.9
RectifiedLinearComponent dim=4096
FullyConnectedComponent input-dim=4096 output-dim=4096 learning-rate=0.02 param-stddev=0.01  bias-stddev=1 weight-decay=0.0005 momentum=0.9
RectifiedLinearComponent dim=4096
FullyConnectedComponent input-dim=4096 output-dim=3454 learning-rate=0.02 param-stddev=0.01 bias-stddev=1 weight-decay=0.0005 momentum=0.9"""
# (H, W, C, kh, kw, G) of its convolutions, for the flop count
NNET_CONVS = [(40, 21, 1, 40, 4, 128), (1, 18, 128, 1, 3, 128), (1, 16, 128, 1, 3, 256),
              (1, 14, 256, 1, 3, 256), (1, 6, 256, 1, 3, 512), (1, 4, 512, 1, 3, 512)]


def nnet_conv_flop():
    return sum(2 * (H - kh + 1) * (W - kw + 1) * G * kh * kw * C
               for H, W, C, kh, kw, G in NNET_CONVS)


def conv_pass_engines(convs, frames, fam):
    """(pass, algorithmic flop, engine) of every convolution pass of a stack,
    by the library's dispatch rules (price each kernel against
    the engine it runs on).  convs: (H, W, C, kh, kw, G, pad, pooled_after)
    per layer; fam: the kernel-family values (kcnn.get_kernel_family).
      forward: the frame-resident kernel for Kdim <= 64 (f16x3 when fwd_x6 is
        2, unpadded, G <= 128 and Kdim <= 32 -- cnsl-conv-frame.hip
        fwd_arith; fp32 MFMA otherwise), else the implicit GEMM: f16x3 when
        igemm_x6 is 3, or 2 and the call is >= 2^34 flop (cnsl-conv-igemm-x6.hip
        use_f16), bf16x6 for 1 or 2 below the rule, fp32 for 0;
      data gradient: the one-pass frame backward for Kdim <= 31 (bf16x6 with
        bwd_x6, fp32 without), else the implicit GEMM in its gather form
        (flipped kernel over the HW input positions) or, when HW >= 1.25 P,
        its scatter form (a 1x1 convolution over the P output positions),
        with the forward's f16x3 rule on that call's flop;
      weight gradient: the frame backward's (Kdim <= 31), else the wide
        kernel: bf16x6 for wgrad_x6 1 / 2, f16x3 for 3, fp32 for 0.
    Returns the list and the number of f16x3 implicit-GEMM calls."""
    out, f16_calls = [], 0

    def igemm(flop_call):
        f = fam["igemm_x6"]
        if f == 3 or (f == 2 and flop_call >= 2 ** 34):
            return "f16x3"
        return "bf16x6" if f else "fp32"
    for i, (h, w, c, kh, kw, g, pad, _) in enumerate(convs):
        oh, ow = h + 2 * pad - kh + 1, w + 2 * pad - kw + 1
        P, HW, Kdim = oh * ow, h * w, kh * kw * c
        flop = 2 * frames * P * g * Kdim
        if Kdim <= 64:
            eng = "f16x3" if (fam["fwd_x6"] == 2 and pad == 0 and g <= 128 and Kdim <= 32) \
                else "bf16x6" if (fam["fwd_x6"] == 1 and pad == 0 and g <= 128 and Kdim <= 31) \
                else "fp32"
        else:
            eng = igemm(flop)
            f16_calls += eng == "f16x3"
        out.append((f"C{i + 1} forward", flop, eng))
        if Kdim <= 31:
            eb = "bf16x6" if fam["bwd_x6"] else "fp32"
            out += [(f"C{i + 1} data gradient", flop, eb), (f"C{i + 1} weight gradient", flop, eb)]
            continue
        npos = P if HW >= 1.25 * P else HW
        eng = igemm(2 * frames * npos * Kdim * g)
        f16_calls += eng == "f16x3"
        out.append((f"C{i + 1} data gradient", flop, eng))
        wf = fam["wgrad_x6"]
        out.append((f"C{i + 1} weight gradient", flop,
                    "f16x3" if wf == 3 else "bf16x6" if wf else "fp32"))
    return out, f16_calls


def engine_ceiling(passes):
    """The fp32-equivalent ceiling of a mix of passes: total flop over the
    time each pass needs at its own engine's peak (a flop-weighted harmonic
    mean of the engines' ceilings)."""
    tot = sum(f for _, f, _ in passes)
    t = sum(f / ENGINE_PEAK_TFLOPS[e] for _, f, e in passes)
    return tot / t if t else None


# the source of each roofline kernel: a PMC byte count (profiles/
# pmc_traffic.json) is only used while the digest of the source it was taken
# from still matches
KERNEL_SOURCES = {
    "conv_bwd_x6q_kernel": "kaldi-cnn_amd/src/cnslmat/cnsl-conv-x6.hip",
    "conv_bwd_x6_kernel": "kaldi-cnn_amd/src/cnslmat/cnsl-conv-x6.hip",
    "conv_fwd_regs_kernel": "kaldi-cnn_amd/src/cnslmat/cnsl-conv-frame.hip",
    "maxpool_direct_prop_kernel": "kaldi-cnn_amd/src/cnslmat/cnsl-hip-kernels.hip",
    "maxpool_direct_backprop_kernel": "kaldi-cnn_amd/src/cnslmat/cnsl-hip-kernels.hip",
    "gemm_f16x3_kernel": "kaldi-cnn_amd/src/kaldi-lite/cu-gemm-f16x3.hip",
    "gemm_f16x3_fast_kernel": "kaldi-cnn_amd/src/kaldi-lite/cu-gemm-f16x3.hip",
    "pool_colmax_kernel": "kaldi-cnn_amd/src/cnslmat/cnsl-conv-frame.hip",
}


def strip_c_comments(text):
    """C/C++ source without its comments, blank lines and trailing blanks
    (string and character literals kept as they are)."""
    out, i, n = [], 0, len(text)
    while i < n:
        c = text[i]
        if c == "/" and text.startswith("//", i):
            j = text.find("\n", i)
            i = n if j < 0 else j
        elif c == "/" and text.startswith("/*", i):
            j = text.find("*/", i + 2)
            i = n if j < 0 else j + 2
            out.append(" ")
        elif c in "\"'":
            j = i + 1
            while j < n and text[j] != c:
                j += 2 if text[j] == "\\" else 1
            out.append(text[i:j + 1])
            i = j + 1
        else:
            out.append(c)
            i += 1
    lines = ("".join(out)).splitlines()
    return "\n".join(l.rstrip() for l in lines if l.strip())


def kernel_source_files(src):
    """`src` and every repo header it includes, transitively (quoted
    #includes resolved as the Makefile's -I../include -Isrc do)."""
    import re
    dirs = [os.path.join(ROOT, "kaldi-cnn_amd/src"), os.path.join(ROOT, "include")]
    seen, todo = [], [os.path.join(ROOT, src)]
    while todo:
        f = todo.pop(0)
        if f in seen:
            continue
        seen.append(f)
        with open(f) as fh:
            code = strip_c_comments(fh.read())
        for inc in re.findall(r'^\s*#\s*include\s+"([^"]+)"', code, re.M):
            for d in [os.path.dirname(f)] + dirs:
                cand = os.path.normpath(os.path.join(d, inc))
                if os.path.exists(cand):
                    todo.append(cand)
                    break
    return seen


def kernel_source_digest(kernel):
    """sha1 of the code (comments and blank lines stripped) of the .hip file
    that defines `kernel` (name up to '<') and of the repo headers it
    includes, transitively; None for an unknown kernel.  A comment-only edit
    leaves it unchanged."""
    import hashlib
    src = KERNEL_SOURCES.get(kernel.split("<")[0].strip())
    if src is None:
        return None
    h = hashlib.sha1()
    for path in kernel_source_files(src):
        with open(path) as fh:
            h.update(os.path.relpath(path, ROOT).encode() + b"\0")
            h.update(strip_c_comments(fh.read()).encode())
    return h.hexdigest()


def parse_profile(text):
    out = {}
    for line in text.strip().splitlines():
        parts = line.split("\t")
        if len(parts) >= 3:
            out[parts[0]] = (float(parts[1].split()[0]), int(parts[2].split()[0]))
    return out


def cpu_baseline(frames_hint, budget_s=12.0):
    """The reference's CPU path, restated by the C oracle: one full c2 step of
    `frames_hint` frames (at most 4096) on this GPU job's CPU share, and
    bounded samples on one thread and on every CPU of the process's affinity.
    The AddMatMat legs (Conv2D's im2col GEMM, conv2D.cc:138-139; the FC GEMMs,
    nnet-component.cc:1227, :1247, nnet-component-nnet0.cc:1141) run on
    OpenBLAS sgemm, as upstream Kaldi's CPU AddMatMat runs on CBLAS; im2col,
    col2im, the reshapes and the maxpool loops are the reference's own CPU
    branches."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    # 16 threads: this GPU's share of the box's host CPUs.  The box exposes
    # every thread of a shared 8-GPU host (nproc = 256 on a 64-core EPYC); a
    # one-GPU job is allotted 16 (OMP_NUM_THREADS there)
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    threads = max(1, min(16, avail))
    blas = O.use_blas(True)
    O.set_threads(threads)
    r = np.random.default_rng(1)
    legs = ("conv_fwd", "pool_fwd", "fc_fwd", "fc_bwd_update", "pool_bwd", "conv_bwd_update")

    def one_step(n):
        oc = O.Conv(H, W, C, KH, KW, G)
        oc.W = (r.standard_normal((KH * KW * C, G)) * 0.01).astype(np.float32)
        oc.b = (r.standard_normal(G) * 0.5).astype(np.float32)
        op = O.Pool(OH, OW, G, 1, 1, PC)
        of = O.FC(POOL_OUT, FC_OUT)
        of.W = (r.standard_normal((FC_OUT, POOL_OUT)) * 0.01).astype(np.float32)
        of.b = np.ones(FC_OUT, np.float32)
        x = r.standard_normal((n, H * W * C)).astype(np.float32)
        dy = (r.standard_normal((n, FC_OUT)) * 1e-2).astype(np.float32)
        ts = []
        t0 = time.perf_counter()
        y1 = oc.propagate(x); ts.append(time.perf_counter())
        y2 = op.propagate(y1); ts.append(time.perf_counter())
        of.propagate(y2); ts.append(time.perf_counter())
        d2 = of.backprop(y2, dy, update=True); ts.append(time.perf_counter())
        d1 = op.backprop(y1, y2, d2); ts.append(time.perf_counter())
        oc.backprop(x, d1, update=True); ts.append(time.perf_counter())
        split = {k: round(b - a, 4) for k, a, b in zip(legs, [t0] + ts[:-1], ts)}
        return ts[-1] - t0, split

    one_step(8)  # first call: library load, thread pools, page faults

    def sized(budget):
        t_small = one_step(16)[0]
        n = int(max(16, min(frames_hint, 16 * budget / max(t_small, 1e-3))))
        n = max(16, (n // 16) * 16)
        t, _ = one_step(n)
        return n, t

    n = max(8, min(4096, frames_hint))
    t, split = one_step(n)
    # one thread (nnet-train-simple --use-gpu=no) ...
    O.set_threads(1)
    n1, t1 = sized(budget_s / 2)
    # ... and every CPU of the affinity mask (nnet-train-parallel
    # --num-threads, train_conv_dropout.sh:205-208), a short sample: on the
    # GPU box those CPUs belong to the other GPUs' jobs too
    all_cores = None
    if avail > threads:
        O.set_threads(avail)
        na, ta = sized(budget_s / 4)
        all_cores = {"value": round(na / ta, 2), "threads": avail, "sample": f"{na} frames"}

    def c1_forward(reps=3):
        """BASELINE configs[0]: Conv + Maxpool forward, 256 frames."""
        oc = O.Conv(H, W, C, KH, KW, G)
        oc.W = (r.standard_normal((KH * KW * C, G)) * 0.01).astype(np.float32)
        oc.b = (r.standard_normal(G) * 0.5).astype(np.float32)
        op = O.Pool(OH, OW, G, 1, 1, PC)
        x = r.standard_normal((256, H * W * C)).astype(np.float32)
        best = float("inf")
        for _ in range(reps):
            t0 = time.perf_counter()
            op.propagate(oc.propagate(x))
            best = min(best, time.perf_counter() - t0)
        return round(256 / best, 1)

    O.set_threads(1)
    c1_1 = c1_forward()
    O.set_threads(threads)
    c1_n = c1_forward()
    # The reference's threaded CPU trainer (nnet-train-parallel --num-threads,
    # train_conv_dropout.sh:205-208; run_nnet.sh:48-50: 16 threads, minibatch
    # 128): T threads, each running the single-thread step on its own
    # minibatches against ONE shared model (Hogwild: unsynchronised in-place
    # updates, as the reference's threads share their Nnet)
    hog = {"unit": "frames/sec", "minibatch": 128,
           "mode": "Hogwild: T threads x single-threaded C oracle step, one shared model",
           "threads_1": hogwild(O, r, 1, 128, budget_s / 6),
           f"threads_{threads}": hogwild(O, r, threads, 128, budget_s / 4)}
    if avail > threads:
        # every CPU of the affinity mask (shared with the other GPUs' jobs),
        # smaller minibatches so the threads' im2col temporaries stay small
        hog[f"threads_{avail}"] = hogwild(O, r, avail, 32, budget_s / 4)
        hog[f"threads_{avail}_minibatch"] = 32
    O.set_threads(threads)
    O.use_blas(False)
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "")
    except OSError:
        pass
    return {"value": round(n / t, 2), "unit": "frames/sec", "cores": threads,
            "kind": "port",
            "sample": f"{n} frames of the c2 stack, one full fwd+bwd+update step, "
                      f"C oracle (oracle/kcnn_oracle.c) with {threads} threads",
            "blas": f"OpenBLAS 0.3.29 sgemm ({os.path.basename(blas)}, numpy's) for the "
                    "AddMatMat legs; im2col / col2im / reshapes / maxpool as the "
                    "reference's CPU loops (OpenMP)",
            "seconds_per_leg": split,
            "single_thread": {"value": round(n1 / t1, 2), "sample": f"{n1} frames, 1 thread"},
            "all_affinity": all_cores,
            "hogwild": hog,
            "c1_forward": {"unit": "frames/sec", "threads_1": c1_1, f"threads_{threads}": c1_n,
                           "sample": "BASELINE configs[0]: Conv+Maxpool forward, 256 frames, "
                                     "best of 3"},
            "host": {"cpu_model": model, "nproc": os.cpu_count(), "affinity": avail,
                     "threads_note": f"{threads} threads = one GPU's share of the box's "
                                     "host CPUs (the job's allotment)"}}


def hogwild(O, r, nthreads, minibatch, budget_s):
    """Aggregate frames/s of nthreads host threads, each training the c2
    stack on its own minibatches (single-threaded C oracle, OpenBLAS on one
    thread) against one shared model, for about budget_s seconds (every
    thread finishes at least one step).  The oracle's ctypes calls release
    the GIL; the model's arrays are updated in place by every thread."""
    import threading
    import numpy as np
    O.set_threads(1)
    oc = O.Conv(H, W, C, KH, KW, G)
    oc.W = (r.standard_normal((KH * KW * C, G)) * 0.01).astype(np.float32)
    oc.b = (r.standard_normal(G) * 0.5).astype(np.float32)
    op = O.Pool(OH, OW, G, 1, 1, PC)
    of = O.FC(POOL_OUT, FC_OUT)
    of.W = (r.standard_normal((FC_OUT, POOL_OUT)) * 0.01).astype(np.float32)
    of.b = np.ones(FC_OUT, np.float32)
    for c in (oc, of):  # the shared state exists before the threads start
        c._c()
    data = [(r.standard_normal((minibatch, H * W * C)).astype(np.float32),
             (r.standard_normal((minibatch, FC_OUT)) * 1e-2).astype(np.float32))
            for _ in range(nthreads)]
    done = [0] * nthreads
    errors = []
    start = threading.Barrier(nthreads + 1)
    deadline = [0.0]

    def worker(i):
        x, dy = data[i]
        start.wait()
        try:
            while True:
                y1 = oc.propagate(x)
                y2 = op.propagate(y1)
                of.propagate(y2)
                d2 = of.backprop(y2, dy, update=True)
                d1 = op.backprop(y1, y2, d2)
                oc.backprop(x, d1, update=True)
                done[i] += 1
                if time.perf_counter() >= deadline[0]:
                    break
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(repr(e))

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(nthreads)]
    for t in ths:
        t.start()
    t0 = time.perf_counter()
    deadline[0] = t0 + budget_s
    start.wait()
    for t in ths:
        t.join()
    el = time.perf_counter() - t0
    if errors:
        return {"error": errors[0]}
    return round(sum(done) * minibatch / el, 2)


def cpu_baseline_stack(config_text, frames, splice_frames=1, budget_s=8.0):
    """The reference's CPU path for a whole config (c5, nnet.config): the C
    oracle's components built from the config lines with random parameters,
    one fwd + bwd + update step on a small sample of frames, OpenBLAS sgemm
    for the AddMatMat legs; reported per frame and labelled as an
    extrapolation from that sample."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    threads = max(1, min(16, avail))
    O.use_blas(True)
    O.set_threads(threads)
    r = np.random.default_rng(2)

    def build():
        layers = []
        for line in config_text.strip().splitlines():
            t, *kvs = line.split()
            kv = dict(x.split("=", 1) for x in kvs)
            gi = lambda k, d=0: int(kv.get(k, d))
            if t == "ConvolutionComponent":
                c = O.Conv(gi("in-height"), gi("in-width"), gi("in-channel"),
                           gi("kernel-height"), gi("kernel-width"), gi("group"),
                           in_pad_height=gi("in-pad-height"), in_pad_width=gi("in-pad-width"))
                kd = gi("kernel-height") * gi("kernel-width") * gi("in-channel")
                c.W = (r.standard_normal((kd, gi("group"))) * 0.01).astype(np.float32)
                c.b = (r.standard_normal(gi("group")) * 0.5).astype(np.float32)
            elif t == "MaxpoolComponent":
                c = O.Pool(gi("in-height"), gi("in-width"), gi("in-channel"),
                           gi("pool-height-dim"), gi("pool-width-dim"), gi("pool-channel-dim"))
            elif t == "FullyConnectedComponent":
                c = O.FC(gi("input-dim"), gi("output-dim"))
                c.W = (r.standard_normal((gi("output-dim"), gi("input-dim"))) * 0.01
                       ).astype(np.float32)
                c.b = np.ones(gi("output-dim"), np.float32)
            elif t == "RectifiedLinearComponent":
                c = O.ReLU(gi("dim"))
            elif t == "SpliceComponent":
                lc, rc = gi("left-context"), gi("right-context")
                c = O.Splice(gi("input-dim"), tuple(range(-lc, rc + 1)))
            else:
                raise ValueError(t)
            layers.append(c)
        return layers

    def step(n):
        layers = build()
        x = r.standard_normal((n * splice_frames, layers[0].input_dim)).astype(np.float32)
        t0 = time.perf_counter()
        ins = []
        a = x
        for c in layers:
            ins.append(a)
            a = c.propagate(a)
        d = (r.standard_normal(a.shape) * 1e-2).astype(np.float32)
        for c, a_in, a_out in zip(reversed(layers), reversed(ins), reversed(ins[1:] + [a])):
            if isinstance(c, O.Pool):
                d = c.backprop(a_in, a_out, d)
            elif isinstance(c, O.ReLU):
                d = c.backprop(a_out, d)
            elif isinstance(c, O.Splice):
                d = c.backprop(d)
            else:
                d = c.backprop(a_in, d, update=True)
        return time.perf_counter() - t0

    step(4)
    t_small = step(8)
    n = int(max(8, min(frames, 8 * budget_s / max(t_small, 1e-3))))
    n = max(8, (n // 8) * 8)
    t = step(n)
    O.use_blas(False)
    return {"value": round(n / t, 2), "unit": "frames/sec", "cores": threads, "kind": "port",
            "sample": f"{n} frames, one fwd+bwd+update step of the whole config on the C "
                      f"oracle with {threads} threads (OpenBLAS sgemm for AddMatMat); "
                      f"per-frame rate extrapolated from this sample to the "
                      f"{frames}-frame batch"}


def baseline_config(frames_per_gpu, world):
    """Which BASELINE.json config a c2-stack run is (configs[1..3])."""
    if frames_per_gpu * world == 131072 and world > 1:
        return "c4: 131072-frame minibatch sharded over %d GPUs" % world
    if frames_per_gpu == 65536 and world == 1:
        return "c3: 65536 frames, 1 GPU"
    if frames_per_gpu == 16384 and world == 1:
        return "one rank's shard of c4 (16384 frames), 1 GPU"
    if frames_per_gpu == 4096:
        return "c2: 4096-frame batch per GPU (BASELINE metric @%d GPU)" % world
    return "c2 stack, %d frames per GPU" % frames_per_gpu


def dp_report(dist, grads, marks, steps, reps=5):
    """The data-parallel exchange of the timed (profiled) steps: the time the
    compute stream waited for the all-reduces at the end of each step (what
    the overlap did not hide), and the same collectives run alone."""
    import torch
    torch.cuda.synchronize()
    exposed = [b.elapsed_time(e) for (nb, b), (ne, e) in zip(marks[0::2], marks[1::2])
               if nb == "wait_begin" and ne == "wait_end"]
    bufs = [grads[i] for i in grads.large] + \
        ([grads.bucket] if grads.bucket is not None else [])
    dist.barrier()
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    for b in bufs:                              # warm the communicator's paths
        dist.all_reduce(b)
    torch.cuda.synchronize()
    t0.record()
    for _ in range(reps):
        for b in bufs:
            dist.all_reduce(b)
    t1.record()
    torch.cuda.synchronize()
    alone = t0.elapsed_time(t1) / reps
    ranks = torch.ones(1, device="cuda")
    dist.all_reduce(ranks)
    exp_ms = sum(exposed) / max(1, len(exposed))
    return {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
            "ranks_seen": int(ranks.item()),
            "collectives_per_step": grads.num_collectives(),
            "allreduce_bytes_per_step": grads.bytes_per_step(),
            "allreduce_alone_ms_per_step": round(alone, 4),
            "allreduce_exposed_ms_per_step": round(exp_ms, 4),
            "overlap_frac": round(1 - exp_ms / alone, 4) if alone > 0 else None,
            "note": "exposed = stream wait at the end of backprop for the step's "
                    "all-reduces (rank 0, profiled pass); alone = the same collectives "
                    "back to back with nothing else running"}


def launch_ranks(n):
    """Run this script under `python -m torch.distributed.run` with n ranks
    on this node (rendezvous on 127.0.0.1, a free port) as a child process;
    returns its exit status (nonzero when the launch itself fails)."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL
    try:
        rc = subprocess.run(cmd, env=env).returncode
    except OSError as e:
        print(f"bench: cannot start {n} ranks: {e}", file=sys.stderr)
        return 2
    if rc != 0:
        print(f"bench: the {n}-rank run exited with status {rc}", file=sys.stderr)
    return rc if rc > 0 else (1 if rc else 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--frames-per-gpu", type=int, default=4096)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", action="store_true",
                    help="one GPU: capture the step once as a HIP graph and replay it "
                         "(measured slower than host-issued steps at c2: 2.75-2.80 M vs "
                         "2.86 M frames/s; c5 1.6 % faster)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--no-fusion", action="store_true",
                    help="run Conv and Maxpool as separate components")
    ap.add_argument("--store-conv-out", action="store_true",
                    help="fused Conv -> Maxpool also stores the conv output")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (default); gloo = rehearsal on shared GPUs")
    ap.add_argument("--config", default="c2", choices=["c2", "c5", "nnet"],
                    help="c2 (default, BASELINE's metric), the c5 deep stack, or the "
                         "reference's egs/exp/nnet/nnet.config model")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` without a launcher: start the N ranks
        # (one process per GPU) as a child torch.distributed.run, before this
        # process touches the GPU, relay its output (rank 0's JSON line) and
        # exit with its status; never a one-GPU line for an N-GPU request
        raise SystemExit(launch_ranks(args.gpus))

    import torch
    import kcnn
    import kcnn_dp

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dist = None
    # one process per GPU; --dist-backend gloo rehearses the N > 1 path with
    # several ranks sharing the GPUs there are (RCCL needs one GPU per rank).
    # Launched by torch.distributed.run (WORLD_SIZE set) the data-parallel
    # step runs even at world size 1 (RCCL's own path, a no-op reduction);
    # plain `python bench.py` is the single-GPU step
    distributed = "WORLD_SIZE" in os.environ
    device = local_rank % max(1, torch.cuda.device_count()) \
        if args.dist_backend == "gloo" else local_rank
    if distributed:
        import torch.distributed as dist
        torch.cuda.set_device(device)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{device}"))
        else:
            dist.init_process_group(args.dist_backend)
    kcnn.init(device)
    kcnn.set_fusion(0 if args.no_fusion else 2 if args.store_conv_out else 1)
    kcnn.set_randn_seed(20261015)  # identical initial params on every replica

    B = args.frames_per_gpu
    in_rows, in_cols, out_cols = B, H * W * C, FC_OUT
    if args.config == "c5":
        text, stack_flop, _ = c5_config()
        net = kcnn.Nnet(text)
    elif args.config == "nnet":
        net = kcnn.Nnet(NNET_CONFIG)
        stack_flop = nnet_conv_flop()
        in_rows, in_cols, out_cols = 21 * B, 40, 3454  # 21 spliced frames per output frame
    else:
        net = kcnn.Nnet(stack_config())
    gen = torch.Generator(device="cuda")
    gen.manual_seed(20261015 + rank)  # each rank its own shard of frames
    x = torch.randn((in_rows, in_cols), generator=gen, device="cuda")
    # the output derivative in a pitched buffer (rows padded to 16 floats), as
    # a CuMatrix holds it (the reference's CuMatrix: cudaMallocPitch); an
    # unpadded 3454-column nnet.config derivative costs the FC GEMMs a copy
    pitch = (out_cols + 15) // 16 * 16
    # a ring of DY_RING seeded derivatives, each followed by its negation, one
    # per step: the same derivative every step drives the parameters one way
    # (nnet.config's FC layers overflowed after a few dozen steps); the ring
    # keeps every pass in the same steady state
    dy_ring = []
    for _ in range(DY_RING // 2):
        base = torch.randn((B, pitch), generator=gen, device="cuda").mul_(1e-2)
        dy_ring += [base[:, :out_cols], base.neg()[:, :out_cols]]
    step_no = [0]

    grads = kcnn_dp.gradient_buffers(
        net, lambda n: torch.empty(n, device="cuda"))

    marks = []

    def mark(name):
        if profiling_dp:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            marks.append((name, e))

    profiling_dp = False

    def step():
        dy = dy_ring[step_no[0] % DY_RING]
        step_no[0] += 1
        if not dist:
            net.Propagate(x)
            net.Backprop(dy)                     # reference semantics: update in Backprop
            return
        kcnn_dp.dp_train_step(net, x, dy, grads, dist, B * world, mark=mark)

    for _ in range(args.warmup):
        step()

    # --graph, one GPU: the step captured once as a HIP graph and replayed
    # (the same kernels with the same arguments; the caching allocator's
    # blocks are warm, so the capture allocates nothing).  Data-parallel steps
    # (RCCL inside) and a failed capture run the step eagerly.
    graph = None
    graph_mallocs = None
    if not dist and args.graph:
        try:
            gs = torch.cuda.Stream()
            gs.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(gs):
                kcnn.sync_stream()
                step()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=gs, capture_error_mode="relaxed"):
                step()
            g.replay()
            torch.cuda.synchronize()
            graph = g
            # the graph writes into the caching allocator's blocks that the
            # capture step held; freed after it, they stay unused only while
            # nothing allocates: checked around every replay
            graph_mallocs = kcnn.device_malloc_calls()
        except Exception as e:  # noqa: BLE001 -- reported, eager fallback
            print(f"bench: HIP graph capture failed ({e!r}); eager steps", file=sys.stderr)
        kcnn.sync_stream()  # back to the current stream

    def timed(profiled):
        """K steps between barriers + device syncs; max over ranks."""
        kcnn.set_profiling(profiled)
        kcnn.reset_profile()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        replay = graph is not None and not profiled
        if replay and kcnn.device_malloc_calls() != graph_mallocs:
            raise SystemExit("bench: a device allocation since the HIP graph's capture; "
                             "its blocks may be reused, the replays are not safe")
        t0 = time.perf_counter()
        for _ in range(args.steps):
            if replay:
                graph.replay()
            else:
                step()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        kcnn.set_profiling(False)
        pr = parse_profile(kcnn.profile_string()) if profiled else {}
        if dist:
            t = torch.tensor([el], device="cuda", dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el, pr

    # headline: profiling off (no events in the stream); then the same K steps
    # again with hipEvents around every component scope, for the per-kernel
    # times of the roofline
    elapsed, _ = timed(False)
    profiling_dp = True
    kcnn.conv_fix_counts(reset=True)
    elapsed_prof, prof = timed(True)
    fc = kcnn.conv_fix_counts()
    f16_calls_lib = fc[0] / args.steps if fc else None  # f16x3 implicit GEMMs per step
    profiling_dp = False
    dp = dp_report(dist, grads, marks, args.steps) if dist else None

    frames = B * world * args.steps
    value = frames / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    if args.config in ("c5", "nnet"):
        # per-scope milliseconds per step (all layers of a kind together)
        scopes = {k: round(v[0] / args.steps, 4) for k, v in sorted(prof.items())}
        conv_ms = sum(v for k, v in scopes.items() if k.startswith("ConvolutionComponent"))
        conv_flop = 3 * stack_flop * B  # fwd + dgrad + wgrad per frame
        fam = {n: kcnn.get_kernel_family(n) for n in ("fwd_x6", "bwd_x6", "igemm_x6",
                                                        "wgrad_x6")}
        convs = ([(h, w, c, kh, kw, g, pad, False) for kind, (h, w, c, kh, kw, g, pad)
                  in ((k, a) for k, a in C5_LAYERS if k == "conv")]
                 if args.config == "c5" else
                 [(h, w, c, kh, kw, g, 0, False) for h, w, c, kh, kw, g in NNET_CONVS])
        passes, f16_pred = conv_pass_engines(convs, B, fam)
        assert abs(sum(f for _, f, _ in passes) - conv_flop) < 1e-6 * conv_flop
        eng_peak = engine_ceiling(passes)
        mix = {}
        for _, f, e in passes:
            mix[e] = mix.get(e, 0) + f
        if args.config == "nnet":
            metric = "frames/sec fwd+bwd, reference egs/exp/nnet/nnet.config model"
            workload = ("nnet.config: Splice(40,+-10) 6x(Conv+ReLU) Maxpool(1x2x1) "
                        "FC 1024-4096-4096-3454 (+ReLU); no Dropout/Softmax")
        else:
            metric = "frames/sec fwd+bwd, c5 deep Conv/Maxpool stack (BASELINE configs[4])"
            workload = ("c5: C1(40x11x3,8x1,256) P1(3x1x4) C2(11x11x64,4x3,256) "
                        "C3(8x9x256,3x3,pad1,256) P2(2x1x4) C4(4x9x64,4x3,256) FC(1792->1024)")
        if rank == 0:
            result = {
                "metric": metric,
                "value": round(value, 1), "unit": "frames/sec", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "f32",
                "data": "synthetic N(0,1) frames",
                "profiled_ms_per_step": round(elapsed_prof / args.steps * 1e3, 4),
                "hip_graph": graph is not None,
                "config": {"workload": workload, "frames_per_gpu": B,
                           "parallelism": f"dp{world}"},
                "conv": {"ms_per_step": round(conv_ms, 4),
                         "TFLOP/s": round(conv_flop / conv_ms / 1e9, 2) if conv_ms else None,
                         # fp32 work over the ceiling of the engines its passes
                         # run on (per pass, conv_pass_engines)
                         "engine_flop_per_step": mix,
                         "engine_ceiling_tflops": round(eng_peak, 1),
                         "engine_frac": round(conv_flop / conv_ms / 1e9 / eng_peak, 4)
                         if conv_ms else None,
                         "passes": [{"pass": n, "engine": e, "gflop": round(f / 1e9, 3)}
                                    for n, f, e in passes],
                         "f16x3_igemm_calls_per_step": {"predicted": f16_pred,
                                                        "library": f16_calls_lib}},
                "scopes_ms_per_step": scopes,
            }
            if conv_ms:
                # the convolution layers (implicit GEMM, weight gradient, frame
                # kernels) as one MFMA-bound scope: the fp32 work of fwd + dgrad
                # + wgrad over the ceiling of the engines its passes run on
                # (f16x3: f16 dense peak / 3 products, bf16x6: bf16 dense peak /
                # 6, fp32: the fp32 MFMA peak), flop-weighted over the passes
                result["roofline"] = {
                    "kernel": "conv layers (every ConvolutionComponent scope)", "bound": "mfma",
                    "achieved": round(conv_flop / conv_ms / 1e9, 2),
                    "peak": round(eng_peak, 1), "unit": "TFLOP/s",
                    "frac": round(conv_flop / conv_ms / 1e9 / eng_peak, 4),
                    "traffic": None, "algorithmic_flop_per_step": conv_flop,
                    "engine": "mix: " + ", ".join(f"{e} {f / conv_flop:.1%}"
                                                  for e, f in sorted(mix.items())),
                    "note": "peak = the flop-weighted ceiling of the engines the passes run on "
                            "(result.conv.passes); fp32 products run on the f16 / bf16 matrix "
                            "cores from split operands (f16x3: 3 products, bf16x6: 6); the fp32 "
                            f"MFMA peak ({PEAK_FP32_MFMA_TFLOPS} TFLOP/s) bounds only the fp32 "
                            "passes"}
            if dp:
                result["dp"] = dp
            if not args.no_cpu_baseline and world == 1:
                text = NNET_CONFIG if args.config == "nnet" else c5_config()[0]
                result["cpu_baseline"] = cpu_baseline_stack(
                    text, B, splice_frames=21 if args.config == "nnet" else 1)
            line = json.dumps(result)
            print(line, flush=True)
            if args.json_out:
                with open(args.json_out, "w") as f:
                    f.write(line + "\n")
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return

    # Per-kernel averages (HIP events around each launch, timed region).
    def avg(key):
        ms, n = prof.get(key, (0.0, 0))
        # cumulative counts include warm-up-free timed steps only
        return (ms / n) if n else None

    k_fwd = avg("ConvolutionComponent::Propagate")
    k_bwd = avg("ConvolutionComponent::BackpropGradient")
    k_dgrad = avg("ConvolutionComponent::BackpropData")
    k_wgrad = avg("ConvolutionComponent::ComputeGradient")
    k_pool_f = avg("MaxpoolComponent::Propagate")
    k_pool_b = avg("MaxpoolComponent::Backprop")
    k_fwd_pool = avg("ConvolutionComponent::PropagateMaxpool")
    k_pool_bm = avg("MaxpoolComponent::BackpropFromMask")
    k_bwd_pooled = avg("ConvolutionComponent::BackpropPooled")
    k_fc = prof.get("AddMatMat", (0.0, 0))
    kernels = {}
    for name, ms, flop, byts in (
            ("conv_fwd", k_fwd, CONV_FLOP_PER_PASS * B, CONV_BYTES_PER_PASS * B),
            ("conv_bwd_fused", k_bwd, CONV_BWD_FLOP * B, CONV_BWD_BYTES * B),
            ("conv_dgrad", k_dgrad, CONV_FLOP_PER_PASS * B, CONV_BYTES_PER_PASS * B),
            ("conv_wgrad", k_wgrad, CONV_FLOP_PER_PASS * B, CONV_BYTES_PER_PASS * B),
            ("maxpool_fwd", k_pool_f, 0, POOL_FWD_BYTES * B),
            ("maxpool_bwd", k_pool_b, 0, POOL_BWD_BYTES * B),
            ("conv_fwd_maxpool", k_fwd_pool, CONV_FLOP_PER_PASS * B,
             (CONV_POOL_FWD_Y_BYTES if args.store_conv_out else CONV_POOL_FWD_BYTES) * B),
            ("maxpool_bwd_mask", k_pool_bm, 0, POOL_BWD_MASK_BYTES * B),
            ("conv_bwd_pooled", k_bwd_pooled, CONV_BWD_FLOP * B, CONV_BWD_POOLED_BYTES * B)):
        if ms:
            # the roofline that bounds it: the larger of bytes/peak-BW and
            # flops/peak-MFMA (algorithmic work)
            t_hbm = byts / (PEAK_HBM_GBS * 1e6)
            t_mfma = flop / (PEAK_FP32_MFMA_TFLOPS * 1e9) if flop else 0.0
            kernels[name] = {"ms": round(ms, 4), "bytes": byts, "flop": flop,
                             "bound": "mfma" if t_mfma > t_hbm else "hbm",
                             "GB/s": round(byts / ms / 1e6, 1),
                             "hbm_frac": round(byts / ms / 1e6 / PEAK_HBM_GBS, 4),
                             "TFLOP/s": round(flop / ms / 1e9, 2) if flop else None}
    gemm_mode = kcnn.get_kernel_family("gemm")
    # each kernel's fp32 work against the engine it runs on: the f16x3 /
    # bf16x6 split engines reach at most the f16 / bf16 dense peak over
    # their products per fp32 product, so every engine_frac is <= 1
    fam = {n: kcnn.get_kernel_family(n) for n in ("fwd_x6", "bwd_x6", "igemm_x6", "wgrad_x6")}
    split = {2: "f16x3", 1: "bf16x6", 0: "fp32"}
    role_family = {"conv_fwd": "fwd_x6", "conv_fwd_maxpool": "fwd_x6", "conv_bwd_fused": "bwd_x6",
                   "conv_bwd_pooled": "bwd_x6", "conv_dgrad": "igemm_x6", "conv_wgrad": "wgrad_x6"}
    for name, k in kernels.items():
        if not k["flop"]:
            continue
        f = fam[role_family[name]]
        eng = split.get(min(f, 2), "fp32") if name not in ("conv_bwd_fused", "conv_bwd_pooled",
                                                            "conv_dgrad", "conv_wgrad") \
            else ("bf16x6" if f else "fp32")
        k["engine"], k["engine_peak_tflops"] = eng, round(ENGINE_PEAK_TFLOPS[eng], 1)
        k["engine_frac"] = round(k["TFLOP/s"] / ENGINE_PEAK_TFLOPS[eng], 4)
    if k_fc[1]:
        # FullyConnectedComponent's three GEMMs (CuMatrixBase::AddMatMat): the
        # in-house f16x3 kernel (kaldi-lite/cu-gemm-f16x3.hip, 3 f16 products
        # per fp32 product) by default, bf16x6 (cu-gemm-x6.hip, 6 bf16
        # products) with KCNN_GEMM=1, rocBLAS sgemm with KCNN_GEMM=0
        fc_tf = FC_FLOP * B / (k_fc[0] / args.steps) / 1e9
        eng = {2: "f16x3", 1: "bf16x6"}.get(gemm_mode, "fp32")
        kernels["fc_gemms"] = {
            "engine": {2: "f16x3 (cu-gemm-f16x3.hip)", 1: "bf16x6 (cu-gemm-x6.hip)"}.get(
                gemm_mode, "rocBLAS sgemm"),
            "ms_per_step": round(k_fc[0] / args.steps, 4),
            "TFLOP/s": round(fc_tf, 2),
            # the three GEMMs' fp32 work over their engine's ceiling (f16 dense
            # peak / 3 products for f16x3)
            "roofline": {"bound": "mfma", "achieved": round(fc_tf, 2),
                         "peak": round(ENGINE_PEAK_TFLOPS[eng], 1), "unit": "TFLOP/s",
                         "frac": round(fc_tf / ENGINE_PEAK_TFLOPS[eng], 4), "engine": eng,
                         "algorithmic_flop_per_step": FC_FLOP * B}}

    # Dominant hand-written hot-path kernel by time.
    dom = max((k for k in kernels if not k.startswith("fc_")),
              key=lambda k: kernels[k]["ms"], default=None)
    roofline = None
    if dom:
        dk = kernels[dom]
        traffic, traffic_kernel = None, None
        pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        # the counter passes (scripts/gpu_profiles.sh) profile the default c2
        # step; their bytes count only for the same role, frame count and
        # kernel source (a changed kernel makes them stale: traffic null)
        if os.path.exists(pmc) and not (args.no_fusion or args.store_conv_out):
            try:
                ent = json.load(open(pmc)).get(dom, {})
                if ent.get("frames") == B and ent.get("source_sha1") and \
                        ent["source_sha1"] == kernel_source_digest(ent.get("kernel", "")):
                    traffic = ent.get("hbm_bytes_per_launch")
                    traffic_kernel = ent.get("kernel")
            except Exception:
                traffic = None
        if dk["bound"] == "mfma":
            achieved, peak, unit = dk["flop"] / dk["ms"] / 1e9, PEAK_FP32_MFMA_TFLOPS, "TFLOP/s"
        else:
            achieved, peak, unit = dk["bytes"] / dk["ms"] / 1e6, PEAK_HBM_GBS, "GB/s"
        roofline = {"kernel": dom, "bound": dk["bound"], "achieved": round(achieved, 2),
                    "peak": peak, "unit": unit, "frac": round(achieved / peak, 4),
                    "traffic": traffic, "traffic_kernel": traffic_kernel,
                    "algorithmic_bytes_per_launch": dk["bytes"],
                    "algorithmic_flop_per_launch": dk["flop"],
                    "launch_ms": dk["ms"]}
        if dk["bound"] == "mfma" and dk.get("engine"):
            # `frac` prices the fp32 work against the fp32 MFMA peak
            # (north_star's target); this is the same work against the engine
            # the kernel runs on (bf16x6: each fp32 operand split exactly into
            # three bf16 parts, six products kept; f16x3: two f16 planes,
            # three products)
            roofline["engine"] = {"name": dk["engine"], "peak": dk["engine_peak_tflops"],
                                  "unit": "TFLOP/s", "frac": dk["engine_frac"]}

    if rank == 0:
        result = {
            "metric": "frames/sec fwd+bwd, Conv+Maxpool+FC stack, 4096-frame batch @1/2/4/8 GPU",
            "value": round(value, 1), "unit": "frames/sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: N(0,1) fbank-shaped frames, a ring of 4 N(0,1)*1e-2 output "
                    "derivatives and their negations, one per step",
            # the second pass of K steps with hipEvents around each scope
            # (kernel times below come from it)
            "profiled_ms_per_step": round(elapsed_prof / args.steps * 1e3, 4),
            "hip_graph": graph is not None,
            "config": {"workload": "c2: Conv(40x11x3, 8x1, 128) -> Maxpool(1x1x4) -> "
                                   "FC(11616->1024), fwd+bwd+update",
                       "baseline_config": baseline_config(B, world),
                       "frames_per_gpu": B, "global_batch": B * world,
                       "parallelism": f"dp{world}",
                       "conv_maxpool_fusion": not args.no_fusion,
                       "conv_output_stored": args.no_fusion or args.store_conv_out},
            "roofline": roofline,
            "kernels": kernels,
        }
        if dp:
            result["dp"] = dp
        if not args.no_cpu_baseline and world == 1:
            result["cpu_baseline"] = cpu_baseline(B)
        line = json.dumps(result)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""xGMI-aware gradient bucket policy (VERDICT r1 "Next round" #2).

The reference takes DDP's defaults (``ref:dpp.py:39`` -> ``torch/nn/parallel/distributed.py:828-834``):
a 1 MiB first bucket, then 25 MiB buckets, in gradient-ready order. Those numbers were picked
for NVLink/NVSwitch and PCIe; on an 8x MI355X node every GPU has 7 point-to-point xGMI links
(~153 GB/s each) and RCCL's all-reduce spreads its rings over them. The policy below sizes
buckets from a two-term cost model of one all-reduce of S bytes over W ranks::

    t(S) = alpha + 2 (W-1)/W * S / B

* ``alpha``  - fixed cost per RCCL all-reduce launch (kernel launch + ring latency);
* ``B``      - achieved all-reduce BUS bandwidth for large messages, i.e. what RCCL's rings
  sustain over the node, not one link: bounded below by one xGMI link (~153 GB/s, a single ring)
  and above by all seven (~1,071 GB/s).

Where they come from, first match wins: explicit arguments; ``XDDP_RCCL_ALPHA_US`` /
``XDDP_RCCL_BUSBW_GBPS``; the job's own init-time measurement (``distributed/calibrate.py``, run
by the DDP constructor when ``XDDP_COMM_CALIBRATE=1`` — the bench default at N>1 — which times the
communicator at the planned bucket sizes and installs the fit with :func:`set_calibration`); and
only then the unmeasured defaults alpha = 30 us, B = 350 GB/s (RCCL spreading several rings over
the links). :func:`calibration_source` says which one a plan used.

Decisions, in gradient-ready order (the order buckets launch in):

1. **first bucket** = 1 MiB cap, as the reference: the first gradients (the classifier head)
   start the comm stream early. With reach-or-exceed closing a large head tensor still ends
   up alone in it.
2. **middle buckets** = ``max(S_eff, T/16)`` capped at 256 MiB, where ``S_eff`` is the size at
   which ``alpha`` is <= 20 % of ``t(S)`` (``S_eff = 4 alpha B W / (2 (W-1))``, ~24 MB at the
   defaults) and ``T`` the total gradient bytes. ``T/16`` keeps >= ~16 buckets in flight for
   big models, so the exposed tail is <= 1/16 of the comm time, while Llama-3-8B (16 GB of
   bf16 grads) runs 50 launches instead of the reference policy's 162 (each of its 117 MB MLP
   weights overshoots a 25 MiB cap and closes a bucket alone; every launch pays ``alpha``).
3. **tail bucket** = the LAST-launched bucket holds only the trailing gradients up to the
   bytes whose transfer takes a quarter of ``alpha`` (``alpha B W / (8 (W-1))``, ~1.5 MB,
   clamped to [1 MiB, 8 MiB]), so its all-reduce costs ~1.25 alpha. Those gradients (ResNet
   stem + layer1, the transformer embedding) are produced by the last backward kernels, so
   their all-reduce cannot overlap anything: with the reference policy ResNet-50's whole last
   bucket (18 MB of bf16 grads) is exposed (~120 us modelled at 350 GB/s), with the tail cap
   ~40 us. The bytes moved out of the tail join the previous bucket, which launches while the
   compute-heavy early layers are still in backward.

At W=1 nothing is communicated and the policy only changes the bucket layout.

A tail bucket cannot split a tensor: when the last-ready gradient is itself large (Llama-3-8B's
1.05 GB token embedding) the tail IS that tensor and its all-reduce (~5 ms modelled at W=8) cannot
overlap backward. What can run under it is the optimizer: with the overlapped optimizer's
``"tail"`` schedule (``DDP.register_overlapped_optimizer``, the bench default for AdamW configs at
W>1) every other bucket's update is DEFERRED until the tail's collectives are launched, the tail is
all-reduced in chunks (``XDDP_TAIL_CHUNK_MB``, default 64 MiB), and the side stream runs the
deferred updates and then each tail chunk's update as soon as that chunk lands. The GPU then does
the step's optimizer work while the links carry the tail, and at most one chunk's update remains
after the last collective. :func:`tail_report` states the modelled exposed time and which of these
mechanisms the run used.

RCCL knobs (:func:`rccl_env_defaults`): none are forced. RCCL picks its channel count for the
node's topology; an unmeasured cap could cut large-bucket bandwidth on the 7-link mesh. A cap
can be requested explicitly with ``XDDP_RCCL_MAX_CHANNELS`` (exported as ``NCCL_MAX_NCHANNELS``
when the user has not set that), e.g. to leave CUs to the backward kernels once an 8-GPU
measurement shows it pays.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Sequence, Tuple

MiB = 1024 * 1024
DEFAULT_ALPHA_US = 30.0
DEFAULT_BUSBW_GBPS = 350.0
MAX_MID_BYTES = 256 * MiB
MIN_MID_BYTES = 25 * MiB
FIRST_BYTES = 1 * MiB


@dataclass(frozen=True)
class BucketPlan:
    first_bytes: int
    cap_bytes: int
    tail_bytes: int
    policy: str

    def as_dict(self):
        return {"policy": self.policy, "first_bytes": self.first_bytes, "cap_bytes": self.cap_bytes,
                "tail_bytes": self.tail_bytes, "alpha_busbw_source": calibration_source()}


_CALIBRATION = None  # (alpha_us, busbw_GBps) measured by distributed/calibrate.py


def set_calibration(alpha_us: float, busbw_gbps: float) -> None:
    """Install the job's measured alpha / B (identical on every rank: fitted from MAX-reduced timings)."""
    global _CALIBRATION
    _CALIBRATION = (float(alpha_us), float(busbw_gbps))


def clear_calibration() -> None:
    global _CALIBRATION
    _CALIBRATION = None


def calibration_source() -> str:
    if os.environ.get("XDDP_RCCL_ALPHA_US") or os.environ.get("XDDP_RCCL_BUSBW_GBPS"):
        return "env"
    return "measured" if _CALIBRATION is not None else "assumed defaults"


def _alpha_us() -> float:
    v = os.environ.get("XDDP_RCCL_ALPHA_US")
    if v:
        return float(v)
    return _CALIBRATION[0] if _CALIBRATION is not None else DEFAULT_ALPHA_US


def _busbw_gbps() -> float:
    v = os.environ.get("XDDP_RCCL_BUSBW_GBPS")
    if v:
        return float(v)
    return _CALIBRATION[1] if _CALIBRATION is not None else DEFAULT_BUSBW_GBPS


def reference_plan(bucket_cap_mb: float = 25, first_bucket_cap_mb: float = 1) -> BucketPlan:
    return BucketPlan(int(first_bucket_cap_mb * MiB), int(bucket_cap_mb * MiB), 0, "reference")


def xgmi_plan(total_bytes: int, world_size: int, alpha_us: float | None = None,
              busbw_gbps: float | None = None) -> BucketPlan:
    """Bucket caps for one DDP job from (total gradient bytes, world size)."""
    alpha = (alpha_us if alpha_us is not None else _alpha_us()) * 1e-6
    bw = (busbw_gbps if busbw_gbps is not None else _busbw_gbps()) * 1e9
    w = max(2, int(world_size))  # W=1 communicates nothing; size as for a pair
    f = 2.0 * (w - 1) / w
    s_alpha = alpha * bw / f      # bytes whose transfer time equals alpha
    s_eff = 4.0 * s_alpha         # alpha <= 20 % of t(S)
    mid = max(s_eff, total_bytes / 16.0)
    mid = int(min(MAX_MID_BYTES, max(MIN_MID_BYTES, mid)))
    tail = int(min(8 * MiB, max(1 * MiB, s_alpha / 4.0)))
    return BucketPlan(FIRST_BYTES, mid, tail, "xgmi")


def assign(sizes_bytes: Sequence[int], plan: BucketPlan) -> List[List[int]]:
    """Bucket layout (positions into ``sizes_bytes``, given in gradient-ready order) for one dtype.

    Mirrors the native rebuild (``Reducer::assign_rebuilt``): the trailing tensors up to
    ``tail_bytes`` form the last bucket; the rest fill buckets that close once they reach
    their cap (reach-or-exceed), the first with ``first_bytes``, the others with ``cap_bytes``.
    """
    n = len(sizes_bytes)
    k = n
    if plan.tail_bytes > 0 and n >= 2:
        acc = 0
        while k > 1 and acc < plan.tail_bytes:
            k -= 1
            acc += sizes_bytes[k]
    out: List[List[int]] = []
    cur: List[int] = []
    acc = 0
    limit = plan.first_bytes
    for i in range(k):
        cur.append(i)
        acc += sizes_bytes[i]
        if acc >= limit:
            out.append(cur)
            cur, acc, limit = [], 0, plan.cap_bytes
    if cur:
        out.append(cur)
    if k < n:
        out.append(list(range(k, n)))
    return out


def bucket_bytes(sizes_bytes: Sequence[int], layout: List[List[int]]) -> List[int]:
    return [sum(sizes_bytes[i] for i in b) for b in layout]


def exposed_tail_us(sizes: List[int], world_size: int, alpha_us: float | None = None,
                    busbw_gbps: float | None = None) -> float:
    """Modelled time of the last bucket's all-reduce (the part of comm backward cannot hide)."""
    alpha = alpha_us if alpha_us is not None else _alpha_us()
    bw = busbw_gbps if busbw_gbps is not None else _busbw_gbps()
    w = max(2, world_size)
    return alpha + 2.0 * (w - 1) / w * sizes[-1] / (bw * 1e3)


def tail_report(sizes: List[int], plan: BucketPlan, world_size: int, overlapped_optimizer=None,
                tail_chunks: int = 0) -> dict:
    """The tail bucket as built, its modelled exposed all-reduce time, and what hides it.

    ``overlapped_optimizer``: None/False (optimizer.step() after backward), ``"tail"`` (updates
    deferred under the chunked tail all-reduce) or ``"backward"``/True (each bucket's update right
    after its own all-reduce, during backward); ``tail_chunks``: collectives the tail was split into."""
    if not sizes:
        return {}
    if overlapped_optimizer is True:
        overlapped_optimizer = "backward"
    exposed = exposed_tail_us(sizes, world_size) if world_size > 1 else 0.0
    # the tail bucket exceeds its cap (buckets close at the first tensor that reaches the cap, so
    # this means the tail's last tensor alone — or with the tensors before it — overshoots)
    over_cap = plan.tail_bytes > 0 and sizes[-1] > plan.tail_bytes
    if world_size <= 1:
        mitigation = "none needed (one rank: nothing is communicated)"
    elif overlapped_optimizer == "tail":
        mitigation = (f"deferred optimizer: the other buckets' updates run on a side stream concurrently with the "
                      f"tail all-reduce, issued as {max(1, tail_chunks)} chunk(s); each chunk's update follows its "
                      f"own collective")
    elif overlapped_optimizer == "backward":
        mitigation = ("none for the tail: each bucket's update runs during backward right after its own "
                      "all-reduce; the tail all-reduce and the tail's update are exposed")
    elif plan.tail_bytes > 0 and not over_cap:
        mitigation = f"tail cap: the last bucket holds <= {plan.tail_bytes} B"
    else:
        mitigation = "none"
    return {"tail_bytes": int(sizes[-1]), "tail_cap_bytes": int(plan.tail_bytes),
            "tail_over_cap": bool(over_cap), "exposed_tail_us_model": round(exposed, 1),
            "optimizer_schedule": overlapped_optimizer or "after backward", "tail_chunks": int(tail_chunks),
            "mitigation": mitigation}


def rccl_env_defaults(world_size: int, backend: str) -> dict:
    """Export the RCCL knobs the user asked for through XDDP_* variables (nothing is forced);
    returns what was set (reported by bench.py)."""
    if world_size <= 1 or backend != "rccl":
        return {}
    applied = {}
    ch = os.environ.get("XDDP_RCCL_MAX_CHANNELS")
    if ch and "NCCL_MAX_NCHANNELS" not in os.environ:
        os.environ["NCCL_MAX_NCHANNELS"] = ch
        applied["NCCL_MAX_NCHANNELS"] = ch
    return applied


def resolve_plan(policy: str | None, bucket_cap_mb, first_bucket_cap_mb, total_bytes: int, world_size: int,
                 backend: str) -> Tuple[BucketPlan, bool]:
    """Pick the plan. Returns (plan, explicit). An explicit ``bucket_cap_mb`` always means the
    reference semantics with that cap. ``policy=None`` = ``XDDP_BUCKET_POLICY`` or, by default,
    ``xgmi`` on the RCCL backend and ``reference`` elsewhere (the CPU backend mirrors gloo and is
    the parity-test backend)."""
    if bucket_cap_mb is not None:
        return reference_plan(bucket_cap_mb, first_bucket_cap_mb or 1), True
    env_cap = os.environ.get("XDDP_BUCKET_CAP_MB")
    if env_cap:
        return reference_plan(float(env_cap), first_bucket_cap_mb or 1), True
    policy = policy or os.environ.get("XDDP_BUCKET_POLICY") or ("xgmi" if backend == "rccl" else "reference")
    if policy == "reference":
        return reference_plan(25, first_bucket_cap_mb or 1), False
    if policy == "xgmi":
        plan = xgmi_plan(total_bytes, world_size)
        if first_bucket_cap_mb:
            plan = BucketPlan(int(first_bucket_cap_mb * MiB), plan.cap_bytes, plan.tail_bytes, plan.policy)
        return plan, False
    raise ValueError(f"unknown bucket policy {policy!r} (use 'reference' or 'xgmi')")

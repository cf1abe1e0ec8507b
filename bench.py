#!/usr/bin/env python3
"""Benchmark of the kfec hot path: device-resident Reed-Solomon encode + decode on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 20:3|10:3dec|200:55|20:3loss1]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Both forms run one process per GPU: without a launcher's WORLD_SIZE, `--gpus N > 1` spawns the N rank
processes itself (spawn_ranks) before any GPU call; a world that differs from --gpus is an error (exit 2).

Metric (BASELINE.json): "FEC encode+decode GiB/s (device-resident), fec=20:3 kcp_mtu=1440".
One step = encode every group of the batch (K data -> R parity shards) and decode every group with R
data shards erased (selection, per-group m x m inverse, recovery MAC), all on the device with inputs
already resident in HBM.  value = payload bytes (G * K * B per GPU, summed over GPUs) per step / step
time, in GiB/s.  Shard groups are independent, so each rank owns a contiguous range of the global group
space (kcptube_amd.partition.group_range; weak scaling, no collective on the data path; gloo carries only
the timing barrier, the max-reduce and the verification flag).

Also reported (rank 0):
  roofline      the dominant kernel (the encode MAC launch; decode for decode-only configs) from HIP events
                on its stream, plus the whole step (encode + decode algorithmic bytes / ms_per_step) as total
                and read-only fractions of the 8 TB/s spec AND of this box's measured linear-read ceiling
                (tools/libkfec_calib.so, timed in the same run), and against the "mix ceiling": the faster of
                (a) the same launch's reads + writes per group in their ideal streaming form (calib_mix: one
                workgroup per group, contiguous 16-B loads, nt stores, no GF arithmetic) and (b) the product's
                own kernel with its GF arithmetic removed (tools/libkfec_arithfree.so: same grid, loads, stores),
                both timed in the same run; for fec=200:55 (VALU-bound) the byte-MAC rate against the measured
                GF-MAC VALU ceiling of the same instruction mix.  Every rank measures its own GPU's ceilings
                (per_rank carries each rank's fractions).
  cpu_baseline  the reference coder (oracle/_ref, compiled from the reference's own sources) on all usable
                host cores over >= 64k distinct groups: rank 0, at every N, after every rank's GPU work.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "FEC encode+decode GiB/s (device-resident), fec=20:3 kcp_mtu=1440, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
SEED = 0x5EED0001

# name: K, N, B, groups per GPU, erasure pool, erasures (ppm for iid), erasure mode, encode?, workload text
#   erasure mode: 0 = exactly `erasures` ids from [0, pool); 1 = 1 + draw % erasures ids; 2 = i.i.d. loss
CONFIGS = {
    "20:3": (20, 23, 1440, 1 << 20, 20, 3, 0, True,
             "fec=20:3 kcp_mtu=1440, 1M shard groups per GPU, encode + decode with 3 data shards erased"),
    "10:3dec": (10, 13, 1400, 1 << 20, 13, 3, 1, False,
                "fec=10:3 kcp_mtu=1400, 1M groups, decode-only, random 1-3 erasures over all 13 shards"),
    "200:55": (200, 255, 1440, 1 << 18, 200, 55, 0, True,
               "fec=200:55 kcp_mtu=1440, 256k groups, encode + decode with 55 data shards erased"),
    "20:3loss1": (20, 23, 1440, 1 << 20, 23, 10000, 2, True,
                  "fec=20:3 kcp_mtu=1440, 1M groups, encode + decode with i.i.d. 1% loss of every shard "
                  "(a live link: ~82% of the groups lost no data shard)"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="20:3", choices=sorted(CONFIGS))
    p.add_argument("--groups", type=int, default=0, help="override groups per GPU")
    p.add_argument("--pitch", type=int, default=0,
                   help="bytes per shard slot in HBM (default: kcp_mtu, rows back to back; a larger pitch only "
                        "aligns the rows -- same shard bytes, same algorithmic traffic -- and is never the headline)")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    p.add_argument("--cpu-seconds", type=float, default=16.0, help="target CPU-seconds of the baseline sample")
    p.add_argument("--cpu-groups", type=int, default=1 << 16, help="distinct groups of the CPU baseline sample")
    p.add_argument("--rehearsal", action="store_true",
                   help="allow more ranks than visible GPUs (ranks share devices as LOCAL_RANK %% count; also "
                        "KFEC_BENCH_REHEARSAL=1): a test of the partition, never a scaling number")
    return p.parse_args()


def rehearsal_allowed(args) -> bool:
    return bool(args.rehearsal) or os.environ.get("KFEC_BENCH_REHEARSAL", "0") not in ("", "0")


def check_devices(world: int, count: int, rehearsal: bool) -> str | None:
    """None if `world` ranks may run on `count` visible devices, else the refusal message.  One rank per GPU:
    fewer devices than ranks would put several ranks on one GPU and report a scaling number no node measured,
    so it is refused unless the run is an explicit rehearsal."""
    if count < 1:
        return "no GPU visible"
    if world > count and not rehearsal:
        return (f"{world} ranks but only {count} visible GPU(s): one rank per GPU is required "
                f"(pass --rehearsal or KFEC_BENCH_REHEARSAL=1 to share devices on purpose)")
    return None


def usable_cores() -> tuple[int, dict]:
    """Cores this process may run on: the affinity set, capped by a cgroup CPU quota if one is set."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    n = aff if quota is None else max(1, min(aff, int(math.floor(quota + 1e-9))))
    return n, {"affinity_cpus": aff, "cgroup_quota_cpus": quota}


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown CPU"


def cpu_baseline(K, N, B, pool, erase, mode, target_cpu_s, groups, decode_only=False):
    """Reference coder on the host cores, bounded sample.  Test infrastructure (oracle/), used here
    only for the reported CPU baseline -- never for the GPU number."""
    import oracle as orc
    threads, cinfo = usable_cores()
    if orc.RefCoder.available():
        ref = orc.RefCoder()
        kind = "reference"
        run = lambda G, thr, passes: ref.bench_roundtrip(K, N, B, G, pool, erase, mode, thr, passes, SEED,
                                                         decode_only)[:2]
    else:
        o = orc.Oracle()
        kind = "port"
        run = lambda G, thr, passes: o.bench_roundtrip(K, N, B, G, erase, thr, passes, SEED)
    # per-group cost on one core (small sample), then the all-core run sized to ~target CPU-seconds
    g_cal = max(16, min(groups, 1024 if K <= 32 else 64))
    bps_cal, secs_cal = run(g_cal, 1, 1)
    per_group = secs_cal / g_cal
    G = groups
    passes = max(1, int(round(target_cpu_s / max(per_group * G, 1e-6))))
    bps, secs = run(G, threads, passes)
    # one core: ~2 s of the same work on a contiguous slice of the same groups
    g1 = int(max(64, min(G, 2.0 / max(per_group, 1e-9))))
    bps1 = run(g1, 1, 1)[0]
    what = "decode-only" if decode_only else "encode + decode"
    erasure = {0: f"{erase} data shards erased", 1: f"random 1-{erase} of all {N} shards erased",
               2: f"i.i.d. {erase / 1e4:g}% loss of every shard"}[mode]
    return {"value": round(bps / 2**30, 3), "unit": "GiB/s", "cores": threads, "kind": kind,
            "value_1core": round(bps1 / 2**30, 4),
            "value_per_core": round(bps / 2**30 / threads, 4),
            "cpu": cpu_model(), **cinfo,
            "sample": f"{G} distinct groups x {passes} passes of fec={K}:{N-K} B={B} {what} ({erasure}), "
                      f"{secs:.1f} s wall on {threads} threads (one contiguous group range and one fec_code "
                      f"per thread); value_1core: {g1} groups x 1 pass on 1 thread"}


def best_ms(torch, launch, reps=5):
    """Fastest of reps + 1 event-timed launches on the current stream (launch(stream) -> 0 on success), or None."""
    s = torch.cuda.current_stream()
    best = None
    for _ in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        if launch(s.cuda_stream) != 0:
            return None
        e1.record(s)
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    return best


class ArithFree:
    """tools/libkfec_arithfree.so (kcptube_amd/build.py): the product's own sources with every GF multiply-accumulate
    of mac_kernel and syn_kernel replaced by a plain XOR of the shard granules and no table reads -- the same grids
    (XCD spans), prep kernels, loads and stores.  Measurement only (its bytes are wrong): its launch time on the
    bench's own tensors is the ceiling of the product kernel's access pattern, timed in the same run."""

    def __init__(self, K, N):
        path = os.path.join(ROOT, "tools", "libkfec_arithfree.so")
        self.lib = ctypes.CDLL(path) if os.path.exists(path) else None
        self.ctx = ctypes.c_void_p()
        self.last = {}
        if not self.lib:
            return
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        self.lib.kfec_create.argtypes = [sz, sz, ctypes.POINTER(vp)]
        self.lib.kfec_destroy.argtypes = [vp]
        self.lib.kfec_encode_batch.argtypes = [vp, sz, sz, sz, vp, vp, vp]
        self.lib.kfec_decode_workspace_size.argtypes = [vp, sz]
        self.lib.kfec_decode_workspace_size.restype = sz
        self.lib.kfec_decode_batch.argtypes = [vp, sz, sz, sz, vp, vp, vp, vp, vp, vp, vp, vp]
        if self.lib.kfec_create(K, N, ctypes.byref(self.ctx)) != 0:
            self.lib = None

    # occupancy caps tried (KFEC_AF_WAVES: at most n waves per SIMD, by LDS padding; None = the kernel's own): without
    # its GF arithmetic the kernel needs fewer registers and runs more waves than the product, which can be slower
    CAPS = (None, 4, 3, 2)

    def _best(self, torch, launch):
        times = {}
        for cap in self.CAPS:
            if cap is None:
                os.environ.pop("KFEC_AF_WAVES", None)
            else:
                os.environ["KFEC_AF_WAVES"] = str(cap)
            times[cap] = best_ms(torch, launch, reps=3)
        os.environ.pop("KFEC_AF_WAVES", None)
        ok = {k: v for k, v in times.items() if v}
        self.last = {("own" if k is None else f"{k}w"): round(v, 4) for k, v in ok.items()}
        return min(ok.values()) if ok else None

    def encode_ms(self, torch, data, parity, B):
        if not self.lib:
            return None
        G, _, pitch = data.shape
        return self._best(torch, lambda st: self.lib.kfec_encode_batch(self.ctx, G, B, pitch, data.data_ptr(),
                                                                       parity.data_ptr(), st))

    def decode_ms(self, torch, data, parity, present, out, out_idx, status, B, dev):
        if not self.lib:
            return None
        G, _, pitch = data.shape
        ws = torch.empty(max(self.lib.kfec_decode_workspace_size(self.ctx, G), 16), dtype=torch.uint8, device=dev)
        return self._best(torch, lambda st: self.lib.kfec_decode_batch(
            self.ctx, G, B, pitch, data.data_ptr(), parity.data_ptr(), present.data_ptr(), out.data_ptr(),
            out_idx.data_ptr(), status.data_ptr(), ws.data_ptr(), st))

    def close(self):
        if self.lib and self.ctx.value:
            self.lib.kfec_destroy(self.ctx)
            self.ctx = ctypes.c_void_p()


class Calib:
    """tools/libkfec_calib.so: on-box read ceiling and GF-MAC VALU ceiling (measurement only)."""

    def __init__(self):
        path = os.path.join(ROOT, "tools", "libkfec_calib.so")
        self.lib = ctypes.CDLL(path) if os.path.exists(path) else None
        if self.lib:
            self.lib.calib_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
            self.lib.calib_read_bytes.argtypes = [ctypes.c_size_t]
            self.lib.calib_read_bytes.restype = ctypes.c_size_t
            self.lib.calib_issue.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
            self.lib.calib_issue_instructions.argtypes = [ctypes.c_uint32]
            self.lib.calib_issue_instructions.restype = ctypes.c_uint64
            self.lib.calib_mix.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                           ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
            self.has_occ = hasattr(self.lib, "calib_mix_occ")
            if self.has_occ:
                self.lib.calib_mix_occ.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                                   ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
        self.mix_last = {}

    def _time(self, torch, launch, reps=5):
        return best_ms(torch, launch, reps)

    def read_ceiling(self, torch, buf):
        """GB/s of a linear read of `buf` (a device tensor of a few GB)."""
        if not self.lib:
            return None
        sink = torch.zeros(16, dtype=torch.int32, device=buf.device)
        n = buf.numel() * buf.element_size()
        ms = self._time(torch, lambda st: self.lib.calib_read(buf.data_ptr(), n, sink.data_ptr(), st))
        return None if ms is None else self.lib.calib_read_bytes(n) / (ms * 1e-3) / 1e9

    def mix_ceiling(self, torch, src, dst, groups, rbytes, wbytes):
        """GB/s of the ideal streaming form of a launch's byte mix: `groups` x (rbytes read contiguously from
        src + wbytes written to dst), one workgroup per group, no GF arithmetic (tools/calib.hip mix_stream)."""
        if not self.lib:
            return None
        r16, w16 = int(rbytes) // 16 * 16, int(round(wbytes / 16.0)) * 16
        groups = min(int(groups), (src.numel() * src.element_size()) // r16,
                     (dst.numel() * dst.element_size()) // max(w16, 1) if w16 else 1 << 62)
        if groups <= 0 or r16 <= 0:
            return None
        sink = torch.zeros(16, dtype=torch.int32, device=src.device)
        runs = {"own": self._time(torch, lambda st: self.lib.calib_mix(src.data_ptr(), dst.data_ptr(), groups, r16, w16,
                                                                      sink.data_ptr(), st))}
        # also at 4 / 3 / 2 workgroups (waves) per SIMD, LDS-capped: fewer, longer streams, as the product kernels run
        for n in ((4, 3, 2) if self.has_occ else ()):
            pad = 160 * 1024 // (n + 1) + 64
            runs[f"{n}w"] = self._time(torch, lambda st, pad=pad: self.lib.calib_mix_occ(
                src.data_ptr(), dst.data_ptr(), groups, r16, w16, pad, sink.data_ptr(), st), reps=3)
        ok = {k: v for k, v in runs.items() if v}
        self.mix_last = {k: round(groups * (r16 + w16) / (v * 1e-3) / 1e9, 1) for k, v in ok.items()}
        return max(self.mix_last.values()) if ok else None

    def gfmac_ceiling(self, torch, dev, cus):
        """Issue bound of the perm MAC on this box, byte-MACs/s: every SIMD issuing nothing but the permutes and
        XORs of the fastest formulation the product uses, at the rates measured by tools/calib.hip's instruction
        chains (8 waves per SIMD).  The 8-row MAC multiplies two shards per row step (KFEC_MAC_PAIR): 6 v_perm_b32 +
        3 v_bitop3_b32 per 8 byte-MACs per lane, i.e. 3 + 1.5 per 4 -- the returned bound.  self.mac_last also keeps
        the single-shard form's (3 v_perm_b32 + v_bitop3_b32 + v_xor_b32 per 4), which rounds 1-5 reported against.
        An upper bound for any kernel built on these instructions."""
        self.mac_last = {}
        if not self.lib:
            return None
        sink = torch.zeros(16, dtype=torch.int32, device=dev)
        blocks = cus * 8
        secs = []
        for op in range(3):
            ms = self._time(torch, lambda st, op=op: self.lib.calib_issue(op, sink.data_ptr(), blocks, st), reps=3)
            if ms is None:
                return None
            # seconds per wave-instruction on one SIMD
            secs.append(ms * 1e-3 / (self.lib.calib_issue_instructions(blocks) / (4.0 * cus)))
        t_perm, t_bitop3, t_xor = secs
        self.mac_last = {"single": 4 * 64 * 4 * cus / (3 * t_perm + t_bitop3 + t_xor),
                         "paired": 4 * 64 * 4 * cus / (3 * t_perm + 1.5 * t_bitop3)}
        return self.mac_last["paired"]


def device_ident(torch, dev, local_dev: int) -> str:
    """host:PCI location of this rank's GPU (falls back to the device index): distinct GPUs of a job are the
    distinct idents over its ranks, on one node or many."""
    import socket
    p = torch.cuda.get_device_properties(dev)
    bus = getattr(p, "pci_bus_id", None)
    loc = f"{getattr(p, 'pci_domain_id', 0):04x}:{bus:02x}:{getattr(p, 'pci_device_id', 0):02x}" if bus is not None else f"dev{local_dev}"
    return f"{socket.gethostname()}:{loc}"


def per_rank_summary(records: list[dict], value: float, payload_per_rank_step: list[float]) -> dict:
    """Evidence for a multi-GPU line, from every rank's own record (gathered after the timed region):
    distinct devices, and value / (world x rank 0's single-rank-equivalent rate) -- rank 0's own payload per
    step over its own wall time per step -- so a 1->N curve shows whether one GPU (or one host launch queue)
    held the job back.  (This is within one run; the driver computes the cross-N scaling efficiency itself.)"""
    world = len(records)
    r0 = records[0]
    rate0 = payload_per_rank_step[0] / (r0["wall_ms_per_step"] * 1e-3) / 2**30 if r0["wall_ms_per_step"] else None
    slowest = max(records, key=lambda r: r["wall_ms_per_step"])
    return {"devices": len({r["device"] for r in records}),
            "rank0_equivalent_GiBps": round(rate0, 2) if rate0 else None,
            "scaling_efficiency": round(value / (world * rate0), 4) if rate0 else None,
            "slowest_rank": slowest["rank"]}


def rank_groups(groups_per_gpu: int, world: int, rank: int) -> tuple[int, int, int]:
    """(g0, g1, total): this rank's contiguous slice of the global group space (weak scaling:
    total = groups_per_gpu * world, split by kcptube_amd.partition.group_range)."""
    from kcptube_amd.partition import group_range
    total = groups_per_gpu * world
    g0, g1 = group_range(total, world, rank)
    return g0, g1, total


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(cmd: list[str], n: int, poll_s: float = 0.2) -> int:
    """`bench.py --gpus N` started without a launcher: run `cmd` as N rank processes of one node (RANK,
    LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT set as torch.distributed.run sets them) and
    return the first non-zero exit code, else 0.  The parent never imports torch or touches a GPU (the
    ranks are fresh processes, not forks of an initialised one); the children inherit stdout, so rank 0's
    JSON line is the parent's output.  When one rank fails the others are terminated (by handle) instead of
    waiting in a barrier for a peer that is gone."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen(cmd, env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:
                    q.terminate()
        if live:
            time.sleep(poll_s)
    for p in procs:
        p.wait()
    return rc


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU: spawn the ranks before anything touches a device in this process
        sys.exit(spawn_ranks([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher formed a world of {world} ranks", file=sys.stderr)
        sys.exit(2)

    # stdout carries exactly one line, rank 0's JSON: everything else the process writes to fd 1 -- gloo's
    # "[Gloo] Rank r is connected to n peer ranks" at rendezvous, runtime chatter -- goes to stderr
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist

    # (device_count does not initialise the GPU; refuse before the rendezvous and before any device work).
    # Ranks per node (LOCAL_WORLD_SIZE, as torch.distributed.run sets it) against this node's GPUs: a multi-node
    # world of 2 x 4 GPUs is 4 ranks per node on 4 devices, not 8 ranks on 4.
    n_dev = torch.cuda.device_count()
    rehearsal = rehearsal_allowed(args)
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)) or world)
    why = check_devices(local_world, n_dev, rehearsal)
    if why:
        print(f"bench.py: {why}", file=sys.stderr)
        sys.exit(2)

    from kcptube_amd import FecCode
    from kcptube_amd.partition import combine_digests, group_range

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    # one rank per GPU; local % count only matters for a multi-rank rehearsal on a smaller box
    local_dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)

    K, N, B, G, pool, erase, mode, do_enc, workload = CONFIGS[args.config]
    if args.groups and args.groups != G:
        G = args.groups
        workload += f" (--groups override: {G} groups per GPU)"
    R = N - K
    g0, g1, total_groups = rank_groups(G, world, rank)  # this rank's contiguous range of the global groups
    G = g1 - g0
    c = FecCode(K, N)
    pitch = max(args.pitch, B) if args.pitch else B
    if pitch != B:
        workload += f" (shard slots padded to a {pitch}-byte pitch)"
    data = torch.empty((G, K, pitch), dtype=torch.uint8, device=dev)
    par = torch.empty((G, R, pitch), dtype=torch.uint8, device=dev)
    masks = torch.empty((G, 4), dtype=torch.int64, device=dev)
    out = torch.empty((G, R, pitch), dtype=torch.uint8, device=dev)
    idx = torch.empty((G, R), dtype=torch.uint8, device=dev)
    st = torch.empty((G,), dtype=torch.uint8, device=dev)
    ws = c.decode_workspace(G, device=dev)
    c.synth(data, SEED, g0=g0, B=B)
    c.erasure_masks(masks, SEED, pool, erase, mode, g0=g0)
    c.encode_batch(data, par, B=B)  # parity exists before a decode-only step
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream()
    n_ev = args.steps
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(n_ev)]

    def step(i=None):
        if i is not None:
            ev[i][0].record(stream)
        if do_enc:
            c.encode_batch(data, par, B=B)
        if i is not None:
            ev[i][1].record(stream)
        c.decode_batch(data, par, masks, out, idx, st, ws, B=B)
        if i is not None:
            ev[i][2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    local_elapsed = time.perf_counter() - t0  # this rank's own steps, before waiting for the others
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    enc_ms = sum(ev[i][0].elapsed_time(ev[i][1]) for i in range(n_ev)) / n_ev
    dec_ms = sum(ev[i][1].elapsed_time(ev[i][2]) for i in range(n_ev)) / n_ev

    # correctness of what was timed (untimed): every erased data shard recovered bit-exact
    mism = torch.zeros(1, dtype=torch.int64, device=dev)
    c.verify_recovered(data, out, idx, mism, B=B)
    torch.cuda.synchronize()
    n_rec = int((idx != 0xFF).sum().item())
    n_dec = int((idx[:, 0] != 0xFF).sum().item()) if R > 0 else 0  # groups with m > 0 (m = 0 reads nothing)
    # (i.i.d. loss: a group that lost more than R shards has too few shares, status 1, as the reference's {})
    st_ok = int(st.max().item()) <= (1 if mode == 2 else 0)
    ok = int(mism.item()) == 0 and st_ok and n_rec > 0
    # KFEC_BENCH_DIGEST=P (tests): the global group space cut into P parts (group_range), one SHA-256 per part
    # over its parity, recovered bytes and recovered ids, gathered in part order and combined (a checksum of
    # checksums): equal for every world size that divides P iff no group was lost, duplicated or changed
    parts = int(os.environ.get("KFEC_BENCH_DIGEST", "0") or 0)
    my_digs = []
    if parts:
        import hashlib
        if parts % world:
            raise SystemExit("KFEC_BENCH_DIGEST must be a multiple of the world size")
        o = out[..., :B].cpu().numpy()
        ix = idx.cpu().numpy()
        o[ix == 0xFF] = 0
        pn = par[..., :B].cpu().numpy()
        for p in range(rank * parts // world, (rank + 1) * parts // world):
            a, b = group_range(total_groups, parts, p)
            a, b = a - g0, b - g0
            my_digs.append(hashlib.sha256(pn[a:b].tobytes() + o[a:b].tobytes() + ix[a:b].tobytes()).hexdigest())
    counts = torch.tensor([0 if ok else 1, n_rec, n_dec], dtype=torch.int64)
    all_digs = [my_digs]
    if world > 1:
        dist.all_reduce(counts, op=dist.ReduceOp.SUM)
        if parts:
            all_digs = [None] * world
            dist.all_gather_object(all_digs, my_digs)
    ok = int(counts[0].item()) == 0
    n_rec_all, n_dec_all = int(counts[1].item()), int(counts[2].item())

    payload = K * B * total_groups * args.steps
    value = payload / elapsed / 2**30
    ms_per_step = elapsed / args.steps * 1e3

    # roofline: algorithmic HBM bytes per launch / measured launch duration (this rank's share)
    enc_bytes = G * (K + R) * B                    # read K*B, write R*B per group
    dec_bytes = n_dec * K * B + n_rec * B          # read the K selected shares, write the m recovered
    enc_read = G * K * B
    dec_read = n_dec * K * B
    if do_enc:
        dom_bytes, dom_read, dom_ms = enc_bytes, enc_read, enc_ms
        dom_name = "mac_kernel<32,MT,encode> (kfec_encode_batch)"
    else:
        dom_bytes, dom_read, dom_ms = dec_bytes, dec_read, dec_ms
        dom_name = "decode_prep + syn_kernel (kfec_decode_batch)"
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    achieved_read = dom_read / (dom_ms * 1e-3) / 1e9
    step_bytes = (enc_bytes if do_enc else 0) + dec_bytes
    step_read = (enc_read if do_enc else 0) + dec_read
    step_ms_local = ms_per_step  # whole step, wall clock, all launches and gaps included
    step_gbs = step_bytes / (step_ms_local * 1e-3) / 1e9
    step_read_gbs = step_read / (step_ms_local * 1e-3) / 1e9

    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            with open(pmc) as f:
                tr = json.load(f).get(args.config if pitch == B else f"{args.config}@p{pitch}")
            if tr and tr.get("groups") == G and tr.get("pitch", B) == pitch:
                traffic = tr.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    # ceilings, measured on EVERY rank's own GPU after the timed region and the verification (the buffers they
    # write -- out, idx, st -- have been checked already): the linear-read ceiling, the ideal streaming form of the
    # dominant launch's byte mix (calib_mix), and the product's own kernels with the GF arithmetic removed
    # (tools/libkfec_arithfree.so: same grid, loads and stores); the mix ceiling is the faster of the two
    calib = Calib()
    read_ceiling = calib.read_ceiling(torch, data)
    if do_enc:
        mix_r, mix_w, mix_g = K * B, R * B, G
    else:
        mix_r, mix_w, mix_g = K * B, (n_rec * B / n_dec if n_dec else 0), max(n_dec, 1)
    mix_calib = calib.mix_ceiling(torch, data, out, mix_g, mix_r, mix_w) if args.config != "200:55" else None
    af = ArithFree(K, N)
    if do_enc:
        af_ms = af.encode_ms(torch, data, out, B)
    else:
        af_ms = af.decode_ms(torch, data, par, masks, out, idx, st, B, dev)
    af.close()
    af_rate = dom_bytes / (af_ms * 1e-3) / 1e9 if af_ms else None
    mix_ceiling = max(mix_calib or 0.0, af_rate or 0.0) or None
    roof = {"bound": "hbm", "kernel": dom_name, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "algorithmic_bytes_per_launch": dom_bytes, "avg_launch_ms": round(dom_ms, 4),
            "achieved_read": round(achieved_read, 1), "frac_read": round(achieved_read / HBM_PEAK_GBS, 4),
            # the whole step (encode + decode) against the spec peak and the measured read ceiling
            "step_bytes": step_bytes, "step_read_bytes": step_read, "step_ms": round(step_ms_local, 4),
            "step_achieved": round(step_gbs, 1), "step_frac": round(step_gbs / HBM_PEAK_GBS, 4),
            "step_frac_read": round(step_read_gbs / HBM_PEAK_GBS, 4),
            "read_ceiling": round(read_ceiling, 1) if read_ceiling else None,
            "step_frac_of_ceiling": round(step_gbs / read_ceiling, 4) if read_ceiling else None,
            "step_frac_read_of_ceiling": round(step_read_gbs / read_ceiling, 4) if read_ceiling else None,
            "frac_of_ceiling": round(achieved / read_ceiling, 4) if read_ceiling else None,
            # the same launch against the faster of two ideal forms of its own read + write mix, both timed in this
            # run: calib_mix (one workgroup per group, contiguous, no arithmetic) and the arithmetic-free build of the
            # product kernel itself (best of 5 launches; the product's time is the mean over the timed steps)
            "mix_ceiling": round(mix_ceiling, 1) if mix_ceiling else None,
            "mix_ceiling_kind": (None if not mix_ceiling else
                                 "arithfree" if (af_rate or 0) >= (mix_calib or 0) else "calib_mix"),
            "mix_ceiling_calib": round(mix_calib, 1) if mix_calib else None,
            "arithfree_ms": round(af_ms, 4) if af_ms else None,
            "arithfree_ms_by_occupancy": af.last, "mix_calib_GBps_by_occupancy": calib.mix_last,
            "arithfree_GBps": round(af_rate, 1) if af_rate else None,
            "mix_ceiling_bytes_per_group": [mix_r, round(mix_w, 1)],
            "frac_of_mix_ceiling": round(achieved / mix_ceiling, 4) if mix_ceiling else None}
    if args.config == "200:55":
        # VALU-bound: byte-MACs per second of each kernel against the perm MAC's issue bound on this box
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        ceil_mac = calib.gfmac_ceiling(torch, dev, cus)
        enc_mac = G * R * K * B / (enc_ms * 1e-3)
        dec_mac = n_rec * K * B / (dec_ms * 1e-3)
        roof.update({"bound": "valu", "unit": "byte-MAC/s", "achieved": round(enc_mac, 0),
                     "peak": round(ceil_mac, 0) if ceil_mac else None,
                     "frac": round(enc_mac / ceil_mac, 4) if ceil_mac else None,
                     "decode_achieved": round(dec_mac, 0),
                     "decode_frac": round(dec_mac / ceil_mac, 4) if ceil_mac else None,
                     "hbm_achieved": round(achieved, 1), "hbm_frac": round(achieved / HBM_PEAK_GBS, 4),
                     "ceiling_kernel": "issue bound of the paired perm MAC: 8 byte-MACs per lane per (6 v_perm_b32 + "
                                       "3 v_bitop3_b32) at the rates tools/calib.hip measures on this box",
                     "issue_bound_single": round(calib.mac_last["single"], 0) if calib.mac_last else None,
                     "frac_of_single_bound": (round(enc_mac / calib.mac_last["single"], 4)
                                              if calib.mac_last else None)})

    # every rank's own timing, device and fractions, gathered after the timed region (per_rank in the JSON line)
    my_rec = {"rank": rank, "device": device_ident(torch, dev, local_dev), "name": torch.cuda.get_device_name(dev),
              "groups": G, "encode_ms": round(enc_ms, 4) if do_enc else None, "decode_ms": round(dec_ms, 4),
              "wall_ms_per_step": round(local_elapsed / args.steps * 1e3, 4),
              "frac": roof["frac"], "frac_of_ceiling": roof["frac_of_ceiling"],
              "frac_of_mix_ceiling": roof["frac_of_mix_ceiling"], "read_ceiling": roof["read_ceiling"],
              "mix_ceiling": roof["mix_ceiling"]}
    records = [my_rec]
    if world > 1:
        records = [None] * world
        dist.all_gather_object(records, my_rec)
    devices = len({r["device"] for r in records})  # distinct GPUs over every rank (and node)

    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": devices,  # distinct GPUs (= ranks, except in a --rehearsal on a smaller box)
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: splitmix64 counter bytes generated on device (SURVEY 8d); erasure patterns per-group PRNG",
        "config": {"workload": workload, "fec": f"{K}:{R}", "kcp_mtu": B, "pitch": pitch, "groups_per_gpu": G,
                   "global_groups": total_groups,
                   "parallelism": f"{world} independent group ranges (no collective)",
                   "ranks": world, "devices": devices, "rehearsal": world > devices},
        "roofline": roof,
        "encode_ms": round(enc_ms, 4) if do_enc else None,
        "decode_ms": round(dec_ms, 4),
        "decode_hbm_GBps": round(dec_bytes / (dec_ms * 1e-3) / 1e9, 1),
        "roundtrip_hbm_GBps": round(((enc_bytes if do_enc else 0) + dec_bytes) / ((enc_ms if do_enc else 0) + dec_ms) / 1e6, 1),
        "recovered_shards_per_step": n_rec_all,
        "decoded_groups_per_step": n_dec_all,
        "verified_bit_exact": ok,
        "cpu_baseline": None,
    }
    if world > 1:
        result["per_rank"] = records
        result["multi_rank"] = per_rank_summary(records, value, [K * B * r["groups"] for r in records])
    if parts:
        result["combined_digest"] = combine_digests([d for ds in all_digs for d in ds])
    if world > 1:
        dist.barrier()  # every rank is past its GPU work: the CPU leg below cannot perturb any GPU timing
    if rank == 0 and not args.no_cpu:
        # the reference coder on this node's host cores, in the same run, at every N (north_star): rank 0 only,
        # after the timed region and every rank's ceilings
        try:
            result["cpu_baseline"] = cpu_baseline(K, N, B, pool, erase, mode, args.cpu_seconds, args.cpu_groups,
                                                  decode_only=not do_enc)
        except Exception as e:  # the GPU number stands on its own
            result["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(result), file=json_out, flush=True)
    if world > 1:
        dist.barrier()  # (the other ranks wait for rank 0's CPU leg instead of tearing the group down under it)
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()

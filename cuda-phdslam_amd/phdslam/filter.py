"""PHDFilter — Python handle on one device-resident particle store.

Mirrors the reference's operator surface (src/phdfilter.h:10-34) over the
C-ABI: set_config ~ setDeviceConfig, predict ~ phdPredict, update ~
phdUpdateSynth, normalize/neff/resample ~ the run_synth loop body
(main.cpp:1233-1297), expected_pose/cardinalities ~ recoverSlamState
(main.cpp:318-388).  All compute happens in libphdslam.so on the GPU.
"""
import ctypes

import numpy as np

from . import _lib
from .types import (ACKERMAN_NOISE, CV_NOISE, GAUSSIAN2D, GAUSSIAN4D, MEASUREMENT, POSE, AckermanControl, Capacity,
                    SlamConfig, csr_from_maps)


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


class PHDFilter:
    def __init__(self, n_particles, config=None, device=0, map_capacity=0, max_measurements=0,
                 candidate_capacity=0, survivor_capacity=0, seed=None, max_particles=0):
        """max_particles: room for the live particles n_predict_particles > 1
        spawns between resamples (default n_particles)."""
        L = _lib.lib()
        cap = Capacity(map_capacity, max_measurements, candidate_capacity, survivor_capacity, max_particles)
        h = ctypes.c_void_p()
        _lib.check(L.phd_ctx_create(ctypes.byref(h), device, n_particles, ctypes.byref(cap)), "phd_ctx_create")
        self._h = h
        self.n_particles = n_particles
        info = Capacity()
        _lib.check(L.phd_ctx_info(h, None, ctypes.byref(info)), "phd_ctx_info")
        self.capacity = info
        self.config = None
        if config is not None:
            self.set_config(config)
        if seed is not None:
            self.set_seed(seed)

    # -- lifecycle -------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().phd_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self):
        return self._h

    @property
    def n(self):
        """Live particles: n_particles, times n_predict_particles per predict until a resample."""
        v = ctypes.c_int()
        _lib.check(_lib.lib().phd_ctx_info(self._h, ctypes.byref(v), None), "phd_ctx_info")
        return v.value

    # -- configuration ---------------------------------------------------
    def set_config(self, cfg: SlamConfig):
        self.config = cfg.copy()
        _lib.check(_lib.lib().phd_set_config(self._h, ctypes.byref(self.config)), "phd_set_config")

    def set_seed(self, seed):
        _lib.check(_lib.lib().phd_set_seed(self._h, int(seed) & (2**64 - 1)), "phd_set_seed")

    def set_stream(self, stream_handle):
        """Enqueue on `stream_handle` (a hipStream_t as int).  0 means the HIP null
        stream (torch's default stream), not the context's private stream."""
        h = ctypes.c_void_p(stream_handle) if stream_handle else ctypes.c_void_p(2**64 - 1)  # PHD_STREAM_NULL
        _lib.check(_lib.lib().phd_set_stream(self._h, h), "phd_set_stream")

    def synchronize(self):
        _lib.check(_lib.lib().phd_synchronize(self._h), "phd_synchronize")

    def set_check_each_update(self, on):
        _lib.check(_lib.lib().phd_set_check_each_update(self._h, 1 if on else 0), "phd_set_check_each_update")

    def set_merge_mode(self, mode):
        """0 = parallel exact greedy merge (serial fallback per particle), 1 = serial greedy only."""
        _lib.check(_lib.lib().phd_set_merge_mode(self._h, int(mode)), "phd_set_merge_mode")

    def set_update_threads(self, threads):
        """Threads per particle of the fused update: 0 = automatic, 256, 512 or 1024."""
        _lib.check(_lib.lib().phd_set_update_threads(self._h, int(threads)), "phd_set_update_threads")

    def update_threads(self):
        """(threads per particle, LDS bytes per workgroup, resident workgroups) of the fused update."""
        t, b, r = ctypes.c_int(), ctypes.c_size_t(), ctypes.c_int()
        _lib.check(_lib.lib().phd_update_threads(self._h, ctypes.byref(t), ctypes.byref(b), ctypes.byref(r)),
                   "phd_update_threads")
        return t.value, b.value, r.value

    def set_update_form(self, form):
        """PHD update form: 0 automatic, 1 one fused launch, 2 split (part A + part C)."""
        _lib.check(_lib.lib().phd_set_update_form(self._h, int(form)), "phd_set_update_form")

    def update_form(self):
        """True when the configured update runs split (part A + part C)."""
        c = ctypes.c_int()
        _lib.check(_lib.lib().phd_update_form(self._h, ctypes.byref(c)), "phd_update_form")
        return bool(c.value)

    def merge_fallbacks(self):
        c = ctypes.c_int()
        _lib.check(_lib.lib().phd_merge_fallbacks(self._h, ctypes.byref(c)), "phd_merge_fallbacks")
        return c.value

    def merge_pair_overflows(self):
        """Particle-updates whose culled pair list overflowed (walked again with the
        exact distances in place) since the last call."""
        c = ctypes.c_int()
        _lib.check(_lib.lib().phd_merge_pair_overflows(self._h, ctypes.byref(c)), "phd_merge_pair_overflows")
        return c.value

    def status_errors(self):
        """Particle-updates that set a capacity / range error status bit since the last call."""
        c = ctypes.c_int()
        _lib.check(_lib.lib().phd_status_errors(self._h, ctypes.byref(c)), "phd_status_errors")
        return c.value

    def particle_status(self):
        """Per-particle status words of the last update (PHD_ST_* bits)."""
        out = np.zeros(self.n, np.int32)
        _lib.check(_lib.lib().phd_particle_status(self._h, _ptr(out)), "phd_particle_status")
        return out

    def check_errors(self):
        _lib.check(_lib.lib().phd_check_errors(self._h), "phd_check_errors")

    # -- state transfer --------------------------------------------------
    def load(self, poses, log_weights, maps, offsets=None):
        """maps: list of GAUSSIAN2D arrays, or a flat array with offsets."""
        if offsets is None:
            maps, offsets = csr_from_maps(maps)
        poses = np.ascontiguousarray(poses, dtype=POSE)
        lw = np.ascontiguousarray(log_weights, dtype=np.float32)
        maps = np.ascontiguousarray(maps, dtype=GAUSSIAN2D)
        offsets = np.ascontiguousarray(offsets, dtype=np.int32)
        n = len(poses)  # n_particles, or up to capacity.max_particles live particles
        assert len(lw) == n and len(offsets) == n + 1
        _lib.check(_lib.lib().phd_load_particles(self._h, n, _ptr(poses), _ptr(lw), _ptr(maps), _ptr(offsets)),
                   "phd_load_particles")

    def export(self, with_maps=True):
        n = self.n
        poses = np.zeros(n, POSE)
        lw = np.zeros(n, np.float32)
        sizes = np.zeros(n, np.int32)
        _lib.check(_lib.lib().phd_export_particles(self._h, n, _ptr(poses), _ptr(lw), _ptr(sizes)),
                   "phd_export_particles")
        offsets = np.zeros(n + 1, np.int32)
        offsets[1:] = np.cumsum(sizes)
        maps = None
        if with_maps:
            maps = np.zeros(int(offsets[-1]), GAUSSIAN2D)
            _lib.check(_lib.lib().phd_export_maps(self._h, n, _ptr(offsets), _ptr(maps)), "phd_export_maps")
        return poses, lw, maps, offsets

    # -- mixed static + dynamic feature model (feature_model 2) ----------
    def enable_dynamic(self, dyn_capacity):
        """Allocate dynamic (Gaussian4D) maps of dyn_capacity components per particle."""
        _lib.check(_lib.lib().phd_enable_dynamic(self._h, int(dyn_capacity)), "phd_enable_dynamic")

    def load_dynamic(self, maps, offsets):
        """Dynamic maps (flat GAUSSIAN4D + offsets[n+1]); call after load()."""
        maps = np.ascontiguousarray(maps, dtype=GAUSSIAN4D)
        offsets = np.ascontiguousarray(offsets, dtype=np.int32)
        assert len(offsets) == self.n + 1
        _lib.check(_lib.lib().phd_load_dynamic_maps(self._h, self.n, _ptr(maps), _ptr(offsets)),
                   "phd_load_dynamic_maps")

    def export_dynamic(self):
        """(dynamic maps, offsets) of the live particles."""
        sizes = np.zeros(self.n, np.int32)
        _lib.check(_lib.lib().phd_dynamic_sizes(self._h, _ptr(sizes)), "phd_dynamic_sizes")
        offsets = np.zeros(self.n + 1, np.int32)
        offsets[1:] = np.cumsum(sizes)
        maps = np.zeros(max(int(offsets[-1]), 1), GAUSSIAN4D)
        _lib.check(_lib.lib().phd_export_dynamic_maps(self._h, self.n, _ptr(offsets), _ptr(maps)),
                   "phd_export_dynamic_maps")
        return maps[:offsets[-1]], offsets

    def predict_dynamic(self):
        """One predictMapMixed of every dynamic map (each predict_* does this with feature_model 2)."""
        _lib.check(_lib.lib().phd_predict_dynamic(self._h), "phd_predict_dynamic")

    def slab_sizes(self):
        s = np.zeros(self.n, np.int32)
        _lib.check(_lib.lib().phd_slab_sizes(self._h, _ptr(s)), "phd_slab_sizes")
        return s

    # -- filter operations -----------------------------------------------
    def predict_ackerman(self, v_encoder, alpha, noise=None, step=0):
        u = AckermanControl(float(alpha), float(v_encoder))
        nz = None
        if noise is not None:
            nz = np.ascontiguousarray(noise, dtype=ACKERMAN_NOISE)
            assert len(nz) == self.n * self._npp()  # one draw per (spawned) particle
        _lib.check(_lib.lib().phd_predict_ackerman(self._h, u, _ptr(nz), int(step)), "phd_predict_ackerman")

    def predict_cv(self, noise=None, step=0):
        nz = None
        if noise is not None:
            nz = np.ascontiguousarray(noise, dtype=CV_NOISE)
            assert len(nz) == self.n * self._npp()
        _lib.check(_lib.lib().phd_predict_cv(self._h, _ptr(nz), int(step)), "phd_predict_cv")

    def _npp(self):
        return max(1, int(self.config.nPredictParticles)) if self.config is not None else 1

    def set_measurements(self, z):
        z = np.ascontiguousarray(z, dtype=MEASUREMENT)
        _lib.check(_lib.lib().phd_set_measurements(self._h, _ptr(z), len(z)), "phd_set_measurements")

    def update(self, z=None):
        if z is not None:
            self.set_measurements(z)
        _lib.check(_lib.lib().phd_update(self._h), "phd_update")

    def normalize(self, lse_override=None):
        ov = ctypes.byref(ctypes.c_float(lse_override)) if lse_override is not None else None
        _lib.check(_lib.lib().phd_normalize(self._h, ov), "phd_normalize")

    def neff(self):
        v = ctypes.c_float()
        _lib.check(_lib.lib().phd_neff(self._h, ctypes.byref(v)), "phd_neff")
        return v.value

    def resample(self, uniforms=None, step=0, return_indices=True):
        u = None
        if uniforms is not None:
            u = np.ascontiguousarray(uniforms, dtype=np.float64)
            assert len(u) == self.n_particles
        idx = np.zeros(self.n_particles, np.int32) if return_indices else None  # n_particles strata
        _lib.check(_lib.lib().phd_resample(self._h, _ptr(u), int(step), _ptr(idx)), "phd_resample")
        return idx

    def step(self, control=None, do_predict=True, step=0):
        """predict -> update -> normalize -> nEff -> resample-if-needed. Returns (neff, resampled)."""
        u = None
        if control is not None:
            v, alpha = control
            u = ctypes.byref(AckermanControl(float(alpha), float(v)))
        neff = ctypes.c_float()
        rs = ctypes.c_int()
        _lib.check(_lib.lib().phd_step(self._h, u, 1 if do_predict else 0, int(step), ctypes.byref(neff),
                                       ctypes.byref(rs)), "phd_step")
        return neff.value, bool(rs.value)

    def expected_pose(self):
        pose = np.zeros(1, POSE)
        mi = ctypes.c_int()
        _lib.check(_lib.lib().phd_expected_pose(self._h, _ptr(pose), ctypes.byref(mi)), "phd_expected_pose")
        return pose[0], mi.value

    def cardinalities(self):
        cn = np.zeros(self.n, np.float32)
        _lib.check(_lib.lib().phd_cardinalities(self._h, _ptr(cn)), "phd_cardinalities")
        return cn

    def expected_map(self):
        """EAP expected map (recoverSlamState's computeExpectedMap, main.cpp:290-316,
        reduced by gm_reduce.cpp:59-132), computed on the device: Gaussian2D
        array in the reference's emission order."""
        nout = ctypes.c_long()
        cap = int(self.export(with_maps=False)[3][-1]) if self.n else 0
        out = np.zeros(max(cap, 1), GAUSSIAN2D)
        _lib.check(_lib.lib().phd_expected_map(self._h, _ptr(out), cap, ctypes.byref(nout)), "phd_expected_map")
        return out[:nout.value]

    def expected_map_dynamic(self):
        """EAP map of the dynamic (Gaussian4D) maps (exp_map_dynamic, main.cpp:369-371),
        computed on the device: Gaussian4D array in the reference's emission order."""
        nout = ctypes.c_long()
        cap = max(int(np.sum(self.dynamic_sizes())), 1)
        out = np.zeros(cap, GAUSSIAN4D)
        _lib.check(_lib.lib().phd_expected_map_dynamic(self._h, _ptr(out), cap, ctypes.byref(nout)),
                   "phd_expected_map_dynamic")
        return out[:nout.value]

    def dynamic_sizes(self):
        sizes = np.zeros(self.n, np.int32)
        _lib.check(_lib.lib().phd_dynamic_sizes(self._h, _ptr(sizes)), "phd_dynamic_sizes")
        return sizes

    def expected_map_groups(self):
        """Decision rounds of the last expected_map (phd_expected_map_groups)."""
        g = ctypes.c_int()
        _lib.check(_lib.lib().phd_expected_map_groups(self._h, ctypes.byref(g)), "phd_expected_map_groups")
        return g.value

    def last_update_ms(self):
        v = ctypes.c_float()
        _lib.check(_lib.lib().phd_last_update_ms(self._h, ctypes.byref(v)), "phd_last_update_ms")
        return v.value

    def enable_timing(self, max_records, stride=1):
        """HIP events around the updates (a ring of max_records), around every
        stride-th update only when stride > 1."""
        _lib.check(_lib.lib().phd_enable_timing(self._h, int(max_records)), "phd_enable_timing")
        _lib.check(_lib.lib().phd_set_timing_stride(self._h, int(stride)), "phd_set_timing_stride")

    def update_timing(self):
        """(summed ms, count) of the fused update kernels recorded since the last call."""
        ms = ctypes.c_float()
        cnt = ctypes.c_int()
        _lib.check(_lib.lib().phd_update_timing(self._h, ctypes.byref(ms), ctypes.byref(cnt)), "phd_update_timing")
        return ms.value, cnt.value

    def set_replay(self, on=True):
        _lib.check(_lib.lib().phd_set_replay(self._h, 1 if on else 0), "phd_set_replay")

    def lse_parts(self):
        out = np.zeros(2, np.float32)
        _lib.check(_lib.lib().phd_lse_parts(self._h, _ptr(out)), "phd_lse_parts")
        return float(out[0]), float(out[1])

    # device-pointer hooks (multi-GPU)
    def copy_log_weights_to(self, dev_ptr):
        _lib.check(_lib.lib().phd_copy_log_weights(self._h, ctypes.c_void_p(dev_ptr)), "phd_copy_log_weights")

    def set_log_weights_from(self, dev_ptr):
        _lib.check(_lib.lib().phd_set_log_weights(self._h, ctypes.c_void_p(dev_ptr)), "phd_set_log_weights")

    def apply_resample(self, dev_idx_ptr, new_log_weight):
        _lib.check(_lib.lib().phd_apply_resample(self._h, ctypes.c_void_p(dev_idx_ptr), float(new_log_weight)),
                   "phd_apply_resample")

    def global_resample(self, dev_w_all_ptr, n_total, offset, seed, step, dev_parents_ptr):
        neff = ctypes.c_float()
        rs = ctypes.c_int()
        _lib.check(_lib.lib().phd_global_resample(self._h, ctypes.c_void_p(dev_w_all_ptr), int(n_total), int(offset),
                                                  int(seed) & (2**64 - 1), int(step), ctypes.c_void_p(dev_parents_ptr),
                                                  ctypes.byref(neff), ctypes.byref(rs)), "phd_global_resample")
        return neff.value, bool(rs.value)

    def cardinality_distribution(self):
        """CPHD: (n, max_cardinality+1) float32 log cardinality distributions."""
        out = np.zeros((self.n, self.config.maxCardinality + 1), np.float32)
        _lib.check(_lib.lib().phd_cardinality_distribution(self._h, out.ctypes.data_as(ctypes.c_void_p)),
                   "phd_cardinality_distribution")
        return out

    def resample_count(self):
        c = ctypes.c_int()
        _lib.check(_lib.lib().phd_resample_count(self._h, ctypes.byref(c)), "phd_resample_count")
        return c.value

    def predict_update(self, control, step, dev_logw_out_ptr=None, do_predict=True):
        """phd_predict_update: predict (Ackerman `control`=(v, alpha), or CV when
        None) + update; optionally copy the log-weights to a device buffer."""
        u = ctypes.byref(AckermanControl(float(control[1]), float(control[0]))) if control is not None else None
        _lib.check(_lib.lib().phd_predict_update(self._h, u, 1 if do_predict else 0, int(step),
                                                 ctypes.c_void_p(dev_logw_out_ptr or 0)), "phd_predict_update")

    def shard_resample(self, dev_w_all_ptr, world, rank, seed, step, dev_parents_ptr, dev_keep_ptr, dev_send_ptr,
                       dev_recv_rec_ptr, dev_records_ptr, send_capacity, new_log_weight):
        """phd_shard_resample -> (neff, resampled, demand, send_records, recv_records)."""
        # per-step call of the sharded step: the out-parameters are allocated once per world size
        bufs = getattr(self, "_shard_bufs", None)
        if bufs is None or bufs[0] != world:
            bufs = (world, ctypes.c_float(), ctypes.c_int(), (ctypes.c_int * world)(), (ctypes.c_int * world)(),
                    (ctypes.c_int * world)())
            self._shard_bufs = bufs
        _, neff, rs, demand, snd, rcv = bufs
        _lib.check(_lib.lib().phd_shard_resample(
            self._h, ctypes.c_void_p(dev_w_all_ptr), int(world), int(rank), int(seed) & (2**64 - 1), int(step),
            ctypes.c_void_p(dev_parents_ptr), ctypes.c_void_p(dev_keep_ptr), ctypes.c_void_p(dev_send_ptr),
            ctypes.c_void_p(dev_recv_rec_ptr), ctypes.c_void_p(dev_records_ptr), int(send_capacity),
            float(new_log_weight), demand, snd, rcv, ctypes.byref(neff), ctypes.byref(rs)), "phd_shard_resample")
        return neff.value, bool(rs.value), list(demand), list(snd), list(rcv)

    def shard_receive(self, dev_records_ptr, dev_recv_rec_ptr, n_slots, first_slot):
        _lib.check(_lib.lib().phd_shard_receive(self._h, ctypes.c_void_p(dev_records_ptr),
                                                ctypes.c_void_p(dev_recv_rec_ptr), int(n_slots), int(first_slot)),
                   "phd_shard_receive")

    def shard_resample_async(self, dev_w_all_ptr, world, rank, seed, step, dev_parents_ptr, dev_keep_ptr,
                             dev_send_ptr, dev_recv_rec_ptr, dev_blocks_ptr, block_records, dev_ovf_ptr,
                             ovf_capacity, new_log_weight):
        """phd_shard_resample_async: the sharded plan with fixed send blocks, no host wait."""
        _lib.check(_lib.lib().phd_shard_resample_async(
            self._h, ctypes.c_void_p(dev_w_all_ptr), int(world), int(rank), int(seed) & (2**64 - 1), int(step),
            ctypes.c_void_p(dev_parents_ptr), ctypes.c_void_p(dev_keep_ptr), ctypes.c_void_p(dev_send_ptr),
            ctypes.c_void_p(dev_recv_rec_ptr), ctypes.c_void_p(dev_blocks_ptr), int(block_records),
            ctypes.c_void_p(dev_ovf_ptr), int(ovf_capacity), float(new_log_weight)), "phd_shard_resample_async")

    def shard_receive_blocks(self, dev_blocks_ptr, block_records, dev_recv_rec_ptr):
        _lib.check(_lib.lib().phd_shard_receive_blocks(self._h, ctypes.c_void_p(dev_blocks_ptr), int(block_records),
                                                       ctypes.c_void_p(dev_recv_rec_ptr)), "phd_shard_receive_blocks")

    def shard_poll(self, world):
        """phd_shard_poll -> (neff, resampled, demand, send_records, recv_records, pending)."""
        bufs = getattr(self, "_poll_bufs", None)
        if bufs is None or bufs[0] != world:
            bufs = (world, ctypes.c_float(), ctypes.c_int(), ctypes.c_int(), (ctypes.c_int * world)(),
                    (ctypes.c_int * world)(), (ctypes.c_int * world)())
            self._poll_bufs = bufs
        _, neff, rs, pend, demand, snd, rcv = bufs
        _lib.check(_lib.lib().phd_shard_poll(self._h, demand, snd, rcv, ctypes.byref(pend), ctypes.byref(neff),
                                             ctypes.byref(rs)), "phd_shard_poll")
        return neff.value, bool(rs.value), list(demand), list(snd), list(rcv), pend.value

    def shard_receive_overflow(self, dev_ovf_ptr, block_records, dev_recv_rec_ptr):
        _lib.check(_lib.lib().phd_shard_receive_overflow(self._h, ctypes.c_void_p(dev_ovf_ptr), int(block_records),
                                                         ctypes.c_void_p(dev_recv_rec_ptr)),
                   "phd_shard_receive_overflow")

    def update_pending(self, control, step, dev_logw_out_ptr=None, do_predict=True):
        u = ctypes.byref(AckermanControl(float(control[1]), float(control[0]))) if control is not None else None
        _lib.check(_lib.lib().phd_update_pending(self._h, u, 1 if do_predict else 0, int(step),
                                                 ctypes.c_void_p(dev_logw_out_ptr or 0)), "phd_update_pending")

    def set_pair_list_cap(self, pairs):
        """phd_set_pair_list_cap: the merge's culled-pair list cap (0 = the layout's; a test hook)."""
        _lib.check(_lib.lib().phd_set_pair_list_cap(self._h, int(pairs)), "phd_set_pair_list_cap")

    def set_edge_pool(self, pool):
        """phd_set_edge_pool: the merge's edge pool (0 = automatic)."""
        _lib.check(_lib.lib().phd_set_edge_pool(self._h, int(pool)), "phd_set_edge_pool")

    def wait_logw(self, stream_handle):
        """phd_wait_logw: `stream_handle` waits until the enqueued updates' log-weights are final."""
        _lib.check(_lib.lib().phd_wait_logw(self._h, ctypes.c_void_p(stream_handle)), "phd_wait_logw")

    def set_plan_stream(self, stream_handle):
        """phd_set_plan_stream: the sharded plan on this stream, beside part C (None: off)."""
        _lib.check(_lib.lib().phd_set_plan_stream(self._h, ctypes.c_void_p(stream_handle or 0)),
                   "phd_set_plan_stream")

    def set_step_births(self, on):
        """phd_set_step_births: the step's own births of the previous scan (1 on,
        0 off, -1 with the filter type: on for CPHD)."""
        _lib.check(_lib.lib().phd_set_step_births(self._h, int(on)), "phd_set_step_births")

    def step_births(self):
        v = ctypes.c_int()
        _lib.check(_lib.lib().phd_step_births(self._h, ctypes.byref(v)), "phd_step_births")
        return bool(v.value)

    def add_births(self, z):
        """phd_add_births: CPHD births of the measurements z (the previous scan)."""
        z = np.ascontiguousarray(z, MEASUREMENT)
        _lib.check(_lib.lib().phd_add_births(self._h, _ptr(z), len(z)), "phd_add_births")

    def set_index_offset(self, offset):
        _lib.check(_lib.lib().phd_set_index_offset(self._h, int(offset)), "phd_set_index_offset")

    def fill_log_weights(self, value):
        _lib.check(_lib.lib().phd_fill_log_weights(self._h, float(value)), "phd_fill_log_weights")

    def record_bytes(self):
        b = ctypes.c_size_t()
        _lib.check(_lib.lib().phd_record_bytes(self._h, ctypes.byref(b)), "phd_record_bytes")
        return b.value

    def pack(self, dev_src_idx_ptr, count, dev_records_ptr):
        _lib.check(_lib.lib().phd_pack_particles(self._h, ctypes.c_void_p(dev_src_idx_ptr), int(count),
                                                 ctypes.c_void_p(dev_records_ptr)), "phd_pack_particles")

    def unpack(self, dev_records_ptr, dev_dst_idx_ptr, count):
        _lib.check(_lib.lib().phd_unpack_particles(self._h, ctypes.c_void_p(dev_records_ptr),
                                                   ctypes.c_void_p(dev_dst_idx_ptr), int(count)),
                   "phd_unpack_particles")

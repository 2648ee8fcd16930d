"""Host-side API of the MI355X front-end: thin Python over the C ABI (include/ssf_frontend.h).

Tensors are torch CUDA (HIP) tensors; their device pointers and torch's current HIP stream
are handed to libssf_frontend.so.  Nothing here computes front-end results itself.

Mirrors of the reference interfaces:
  Frontend.extract_planes*  <- frameFeature.cpp cloudHandler (:35-139)
  Frontend.plane_table / register  <- lidarOdometry_onlyPC.cpp frameRegistration (:147-252)
                                       + publishResult accumulation (:87-90)
  Frontend.mask_pose        <- PointCloudOdometry_noSeg.py:97-125 / PointCloudOdometry.py:91-101
  OdometryState             <- the cloudThread() state machine (flagStart, warm start, last<-curr,
                               lidarOdometry_onlyPC.cpp:281-311) for many sequences at once
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import torch

from . import _abi
from ._abi import SSFError

SOLVERS = {"ceres_lm": _abi.SOLVER_CERES_LM, "lm": _abi.SOLVER_CERES_LM, "gn": _abi.SOLVER_GN}
MASK_MODES = {"gmm": _abi.MASK_GMM, "gt": _abi.MASK_GT, "given": _abi.MASK_GIVEN}


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream(device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def frame_offsets(counts, device):
    """int64 offsets [F+1] (device) and their host copy from a list of frame sizes."""
    off = [0]
    for c in counts:
        off.append(off[-1] + int(c))
    h = torch.tensor(off, dtype=torch.int64)
    return h.to(device), h


@dataclass
class PlaneBatch:
    """Plane clouds of F frames at frame offsets: xyzi[off[f] : off[f] + count[f]]."""
    xyzi: torch.Tensor      # [total, 4] f32
    count: torch.Tensor     # [F] int32 (device)
    off: torch.Tensor       # [F+1] int64 (device)
    h_off: torch.Tensor     # [F+1] int64 (host)
    max_points: int         # host bound on points per frame (grid sizing)

    def frame(self, f):
        c = int(self.count[f])
        o = int(self.h_off[f])
        return self.xyzi[o:o + c]


class PlaneTable(tuple):
    """(normal, valid, sorted_xyzi, sorted_idx) of ssf_plane_table_batch; .strips = (strip_xyzi,
    strip_head), the y-strip image the association of the next pairs stages, or None."""

    def __new__(cls, normal, valid, sx, si, strips=None):
        t = super().__new__(cls, (normal, valid, sx, si))
        t.strips = strips
        return t

    def tensors(self):
        """every device tensor the table holds (for record_stream across streams)"""
        return [x for x in (*self, *(self.strips or ())) if isinstance(x, torch.Tensor)]


class Frontend:
    """One C-ABI context (one device, one parameter profile)."""

    def __init__(self, n_rows: int = 64, device: int | torch.device | None = None,
                 solver: str = "ceres_lm", max_iter: int | None = None, ring_chain: str = "float"):
        """ring_chain: the evaluation of frameFeature.cpp:57's atan / sqrt -- "float" (the float
        overloads libstdc++'s <math.h> makes visible; the default) or "double" (C's double
        functions only); include/ssf_frontend.h SSF_RING_CHAIN_*."""
        if not torch.cuda.is_available():
            raise SSFError("no HIP device visible: the MI355X front-end has no CPU fallback")
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else
                           (device.index if isinstance(device, torch.device) else int(device)))
        self.device = dev
        self.cfg = _abi.config_default(n_rows)
        self.cfg.solver = SOLVERS[solver]
        self.cfg.max_iter = (8 if self.cfg.solver == _abi.SOLVER_CERES_LM else 10) if max_iter is None else int(max_iter)
        if ring_chain not in _abi.RING_CHAINS:
            raise ValueError(f"ring_chain must be one of {sorted(_abi.RING_CHAINS)}, got {ring_chain!r}")
        self.cfg.ring_chain = _abi.RING_CHAINS[ring_chain]
        self.n_rows = n_rows
        h = C.c_void_p()
        rc = _abi.lib().ssf_create(dev.index, C.byref(self.cfg), C.byref(h))
        if rc != _abi.SSF_OK:
            raise SSFError(f"ssf_create failed rc={rc} (need a gfx950 / MI355X device)")
        self._h = h

    # ------------------------------------------------------------------ plumbing
    def close(self):
        if getattr(self, "_h", None):
            _abi.lib().ssf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != _abi.SSF_OK:
            msg = _abi.lib().ssf_last_error(self._h)
            raise SSFError(f"{what} failed rc={rc}: {msg.decode() if msg else ''}")

    def reserve(self, max_frames: int, max_points_per_frame: int):
        self._check(_abi.lib().ssf_reserve(self._h, max_frames, max_points_per_frame), "ssf_reserve")

    def profile(self, on: bool = True):
        """Bracket every kernel this context launches with HIP events (kernel-only durations
        when the stream runs alone); read them with kernel_times()."""
        self._check(_abi.lib().ssf_profile_enable(self._h, 1 if on else 0), "ssf_profile_enable")

    def kernel_times(self) -> dict:
        """{kernel name: (launches, total ms)} recorded since the previous call (synchronises)."""
        buf = (_abi.KernelTime * 64)()
        n = C.c_int32(0)
        self._check(_abi.lib().ssf_profile_read(self._h, buf, 64, C.byref(n)), "ssf_profile_read")
        return {buf[i].name.decode(): (int(buf[i].launches), float(buf[i].total_ms)) for i in range(n.value)}

    def mask_split(self, parts_per_frame: int = 0):
        """Work-groups per frame of the GMM fit (0 = automatic, 1..32 fixed)."""
        self._check(_abi.lib().ssf_set_mask_split(self._h, int(parts_per_frame)), "ssf_set_mask_split")

    def mask_schedule(self, order=None, queue: int = 0):
        """Frame scheduling of the next mask_pose launches (ssf_set_mask_schedule; outputs do not
        depend on it): order = a device int32 permutation of the batch's frames (dispatch order,
        e.g. longest-first by the previous step's passes; the tensor must outlive the launches
        that read it -- keep a reference), queue = at most this many work-groups taking frame
        tickets (0: one per frame).  mask_schedule() resets both."""
        if order is not None:
            order = self._dev(order, torch.int32)
            if order.dim() != 1 or order.numel() == 0:
                raise ValueError("order must be a non-empty 1-D int32 device tensor")
        self._mask_order = order                   # the context keeps only the pointer
        self._check(_abi.lib().ssf_set_mask_schedule(self._h, _ptr(order), 0 if order is None else order.numel(),
                                                     int(queue)), "ssf_set_mask_schedule")

    def edge_config(self, **kw):
        """Edge-feature parameters (beyond the reference; ssf_set_edge_config): edge_min,
        edge_span, line_ratio, max_nn_d2.  No arguments: the current defaults."""
        ec = _abi.EdgeConfig()
        self._check(_abi.lib().ssf_edge_config_default(self.n_rows, C.byref(ec)), "ssf_edge_config_default")
        for k, v in kw.items():
            if not hasattr(ec, k):
                raise ValueError(f"unknown edge parameter {k!r}")
            setattr(ec, k, v)
        self._check(_abi.lib().ssf_set_edge_config(self._h, C.byref(ec)), "ssf_set_edge_config")
        self._edge_span = int(ec.edge_span)
        return {k: getattr(ec, k) for k, _ in ec._fields_}

    def seed(self, seed: int):
        """np.random.seed(seed) for the GMM's k-means++ RandomState."""
        self._check(_abi.lib().ssf_rng_seed(self._h, seed & 0xFFFFFFFF), "ssf_rng_seed")

    def _dev(self, t, dtype):
        if not (t.is_cuda and t.device == self.device and t.dtype == dtype and t.is_contiguous()):
            raise SSFError(f"expected a contiguous {dtype} tensor on {self.device}")
        return t

    # ------------------------------------------------------------------ frameFeature
    def _out(self, t, shape, dtype, what):
        """a caller-supplied output buffer (preallocated: no allocation per call), checked"""
        t = self._dev(t, dtype)
        if t.dim() != len(shape) or any(a < b for a, b in zip(t.shape, shape)) or t.shape[1:] != shape[1:]:
            raise ValueError(f"{what}: need at least {tuple(shape)} {dtype}, got {tuple(t.shape)}")
        return t

    def extract_planes_batch(self, pts, off, h_off, max_points=None, point_stride=None,
                             debug=False, keep=None, out=None):
        """cloudHandler for F frames packed in `pts` ([total, stride] f32) at offsets `off`.
        Returns PlaneBatch (and, with debug=True, ring-ordered points, row offsets, curvature).
        keep (uint8/bool per point, optional, beyond the reference): extract from the kept
        points only -- e.g. the background mask of mask_pose ("mask applied before features").
        out: optional preallocated (plane [>= total, 4] f32, count [>= F] int32) -- a pipeline
        reuses a ring of them instead of allocating per call."""
        pts = self._dev(pts, torch.float32)
        F = h_off.numel() - 1
        total = int(h_off[-1])
        sizes = (h_off[1:] - h_off[:-1])
        mx = int(sizes.max()) if max_points is None and F > 0 else int(max_points or 0)
        stride = pts.shape[1] if point_stride is None else point_stride
        if out is not None:
            plane = self._out(out[0], (max(total, 1), 4), torch.float32, "plane out")
            count = self._out(out[1], (max(F, 1),), torch.int32, "count out")
        else:
            plane = torch.empty((max(total, 1), 4), dtype=torch.float32, device=self.device)
            count = torch.empty(max(F, 1), dtype=torch.int32, device=self.device)
        ring = roff = curv = None
        if debug:
            ring = torch.zeros((max(total, 1), 4), dtype=torch.float32, device=self.device)
            roff = torch.zeros(max(F, 1) * (self.n_rows + 1), dtype=torch.int32, device=self.device)
            curv = torch.zeros(max(total, 1), dtype=torch.float32, device=self.device)
        if keep is None:
            rc = _abi.lib().ssf_extract_planes_batch(
                self._h, _stream(self.device), F, _ptr(pts), stride, _ptr(off), total, mx,
                _ptr(plane), _ptr(count), _ptr(ring), _ptr(roff), _ptr(curv))
            self._check(rc, "ssf_extract_planes_batch")
        else:
            keep = self._dev(keep, torch.uint8)
            if keep.numel() != total:
                raise ValueError(f"keep has {keep.numel()} entries for {total} points")
            rc = _abi.lib().ssf_extract_planes_batch_masked(
                self._h, _stream(self.device), F, _ptr(pts), stride, _ptr(off), total, mx, _ptr(keep),
                _ptr(plane), _ptr(count), _ptr(ring), _ptr(roff), _ptr(curv))
            self._check(rc, "ssf_extract_planes_batch_masked")
        # plane points per frame <= sum over rows of ceil(n_r / planeSpan) <= n/span + rows
        # out= buffers may be larger than this call needs: hand on the first max(total, 1) rows
        # (a view), so downstream sizes (plane_table, register_chain) follow the real point count
        pb = PlaneBatch(plane[:max(total, 1)], count[:F], off, h_off,
                        min(mx, mx // max(1, self.cfg.plane_span) + self.n_rows + 1))
        if debug:
            return pb, ring, roff.view(max(F, 1), self.n_rows + 1)[:F], curv
        return pb

    def extract_features_batch(self, pts, off, h_off, max_points=None, keep=None, out=None):
        """extract_planes_batch plus the edge cloud (beyond the reference: edge features,
        ssf_extract_features_batch) -> (planes PlaneBatch, edges PlaneBatch).
        out: optional preallocated (plane [>= total, 4], count [>= F], edge [>= total, 4],
        ecount [>= F])."""
        pts = self._dev(pts, torch.float32)
        F = h_off.numel() - 1
        total = int(h_off[-1])
        sizes = (h_off[1:] - h_off[:-1])
        mx = int(sizes.max()) if max_points is None and F > 0 else int(max_points or 0)
        if out is not None:
            plane = self._out(out[0], (max(total, 1), 4), torch.float32, "plane out")
            count = self._out(out[1], (max(F, 1),), torch.int32, "count out")
            edge = self._out(out[2], (max(total, 1), 4), torch.float32, "edge out")
            ecount = self._out(out[3], (max(F, 1),), torch.int32, "edge count out")
        else:
            plane = torch.empty((max(total, 1), 4), dtype=torch.float32, device=self.device)
            count = torch.empty(max(F, 1), dtype=torch.int32, device=self.device)
            edge = torch.empty((max(total, 1), 4), dtype=torch.float32, device=self.device)
            ecount = torch.empty(max(F, 1), dtype=torch.int32, device=self.device)
        if keep is not None:
            keep = self._dev(keep, torch.uint8)
            if keep.numel() != total:
                raise ValueError(f"keep has {keep.numel()} entries for {total} points")
        rc = _abi.lib().ssf_extract_features_batch(
            self._h, _stream(self.device), F, _ptr(pts), pts.shape[1], _ptr(off), total, mx,
            _ptr(keep), _ptr(plane), _ptr(count), _ptr(edge), _ptr(ecount))
        self._check(rc, "ssf_extract_features_batch")
        span = getattr(self, "_edge_span", None) or (10 if self.n_rows == 64 else 3)
        pb = PlaneBatch(plane[:max(total, 1)], count[:F], off, h_off,
                        min(mx, mx // max(1, self.cfg.plane_span) + self.n_rows + 1))
        eb = PlaneBatch(edge[:max(total, 1)], ecount[:F], off, h_off, min(mx, mx // max(1, span) + self.n_rows + 1))
        return pb, eb

    def edge_table(self, eb: PlaneBatch, out=None):
        """Line table of frames that will be LAST frames (beyond the reference):
        -> (line [total, 6] f32: centroid, direction; valid [total] u8).
        out: optional preallocated (line, valid)."""
        total = eb.xyzi.shape[0]
        if out is not None:
            line = self._out(out[0], (total, 6), torch.float32, "line out")
            valid = self._out(out[1], (total,), torch.uint8, "line valid out")
        else:
            line = torch.empty((total, 6), dtype=torch.float32, device=self.device)
            valid = torch.empty(total, dtype=torch.uint8, device=self.device)
        rc = _abi.lib().ssf_edge_table_batch(self._h, _stream(self.device), eb.count.numel(),
                                             _ptr(eb.xyzi), _ptr(eb.off), _ptr(eb.count),
                                             eb.max_points, _ptr(line), _ptr(valid))
        self._check(rc, "ssf_edge_table_batch")
        return line, valid

    def extract_planes(self, pts, xyz_offset: int = 0):
        """Single frame, PointCloud2-style points [n, k] f32 (point_step = 4k bytes, x/y/z at
        byte offsets xyz_offset + 0/4/8) -> plane cloud [m, 4]."""
        pts = self._dev(pts, torch.float32)
        n = pts.shape[0]
        out = torch.empty((max(n, 1), 4), dtype=torch.float32, device=self.device)
        m = C.c_int64(0)
        rc = _abi.lib().ssf_extract_planes(self._h, _stream(self.device), _ptr(pts), n,
                                           4 * pts.shape[1], int(xyz_offset), _ptr(out), C.byref(m), n)
        self._check(rc, "ssf_extract_planes")
        return out[:m.value]

    # ------------------------------------------------------------------ lidarOdometry_onlyPC
    def plane_table(self, pb: PlaneBatch, brute_force: bool = False, strips: bool = True, out=None):
        """-> PlaneTable (normal [total,3] f32, valid [total] u8, sorted_xyzi, sorted_idx) -- the
        plane table of frames that will be LAST frames, plus their x-sorted search index (None,
        None when brute_force=True); .strips = the y-strip image (strip_xyzi [total,4] f32,
        strip_head [total] i32) that register() hands to the association, or None.
        out: optional preallocated buffers (normal, valid, sx, si, strip_xyzi, strip_head), each
        at least `total` rows -- reused instead of allocated per call."""
        total = pb.xyzi.shape[0]
        if out is not None:
            normal = self._out(out[0], (total, 3), torch.float32, "normal out")
            valid = self._out(out[1], (total,), torch.uint8, "valid out")
        else:
            normal = torch.empty((total, 3), dtype=torch.float32, device=self.device)
            valid = torch.empty(total, dtype=torch.uint8, device=self.device)
        sx = si = st = None
        if not brute_force:
            if out is not None:
                sx = self._out(out[2], (total, 4), torch.float32, "sorted_xyzi out")
                si = self._out(out[3], (total,), torch.int32, "sorted_idx out")
            else:
                sx = torch.empty((total, 4), dtype=torch.float32, device=self.device)
                si = torch.empty(total, dtype=torch.int32, device=self.device)
            # the association stages an image only for frames of STRIP_IMAGE_MIN..MAX points
            # (registration.hip strip_image_frame) and only in launches whose plane bound is
            # within MAX (float4 strips): otherwise the 20 B per plane point would be dead weight
            if strips and _abi.STRIP_IMAGE_MIN <= pb.max_points and pb.max_points <= _abi.STRIP_IMAGE_MAX:
                if out is not None:
                    st = (self._out(out[4], (total, 4), torch.float32, "strip_xyzi out"),
                          self._out(out[5], (total,), torch.int32, "strip_head out"))
                else:
                    st = (torch.empty((total, 4), dtype=torch.float32, device=self.device),
                          torch.empty(total, dtype=torch.int32, device=self.device))
        rc = _abi.lib().ssf_plane_table_batch(self._h, _stream(self.device), pb.count.numel(),
                                              _ptr(pb.xyzi), _ptr(pb.off), _ptr(pb.count),
                                              pb.max_points, _ptr(normal), _ptr(valid), _ptr(sx),
                                              _ptr(si), _ptr(st[0] if st else None),
                                              _ptr(st[1] if st else None))
        self._check(rc, "ssf_plane_table_batch")
        return PlaneTable(normal, valid, sx, si, st)

    def register_pair(self, last_xyzi, curr_xyzi, q_init=(0.0, 0.0, 0.0, 1.0),
                      t_init=(0.0, 0.0, 0.0)):
        """frameRegistration() for one pair with the reference's globals as arguments
        (ssf_register_pair): plane clouds [m, 4] f32 on the device, warm start para_q (x,y,z,w)
        / para_t -> (q, t, steps, n_corr); steps = per-iteration dicts (pose, cost, status,
        radius); n_corr = -1 when the last frame has <= 10 points (:158)."""
        last_xyzi = self._dev(last_xyzi, torch.float32)
        curr_xyzi = self._dev(curr_xyzi, torch.float32)
        if last_xyzi.dim() != 2 or last_xyzi.shape[1] != 4 or curr_xyzi.dim() != 2 or curr_xyzi.shape[1] != 4:
            raise ValueError("plane clouds must be [m, 4] (x, y, z, intensity)")
        qi = (C.c_double * 4)(*[float(v) for v in q_init])
        ti = (C.c_double * 3)(*[float(v) for v in t_init])
        qo, to = (C.c_double * 4)(), (C.c_double * 3)()
        cap = max(1, int(self.cfg.max_iter))
        steps = (_abi.Step * cap)()
        log = _abi.StepLog(cap, 0, 0, 0, steps)
        rc = _abi.lib().ssf_register_pair(self._h, _stream(self.device), _ptr(last_xyzi),
                                          last_xyzi.shape[0], _ptr(curr_xyzi), curr_xyzi.shape[0],
                                          qi, ti, qo, to, C.byref(log))
        self._check(rc, "ssf_register_pair")
        out = [dict(q=list(steps[i].q), t=list(steps[i].t), cost=steps[i].cost,
                    status=_abi.STEP_STATUS.get(steps[i].status, steps[i].status),
                    radius=steps[i].radius) for i in range(log.n_steps)]
        return list(qo), list(to), out, int(log.n_corr)

    def register_chain(self, pb: PlaneBatch, table, pose_init, pose_abs_init=None, out=None,
                       want_ncorr=False):
        """frameRegistration over a sequence (ssf_register_chain): pair k registers frame k + 1 of
        pb against frame k, warm-started from pair k - 1's solution (pose_init [7] or [1, 7] for
        pair 0; lidarOdometry_onlyPC.cpp:164,251-252).  table = plane_table(pb).  Returns
        dict(pose_seq [K, 7], pose_abs_seq [K, 7] (frame k + 1's pose from pose_abs_init) or None,
        ncorr [K] or None); out: optional preallocated pose_seq."""
        F = pb.count.numel()
        K = max(F - 1, 0)
        pose_init = self._dev(pose_init, torch.float64).reshape(-1)
        if pose_init.numel() != 7:
            raise ValueError("pose_init must hold 7 values (q xyzw, t)")
        seq = self._out(out, (max(K, 1), 7), torch.float64, "pose_seq out") if out is not None else \
            torch.empty((max(K, 1), 7), dtype=torch.float64, device=self.device)
        abs_seq = None
        if pose_abs_init is not None:
            pose_abs_init = self._dev(pose_abs_init, torch.float64).reshape(-1)
            if pose_abs_init.numel() != 7:
                raise ValueError("pose_abs_init must hold 7 values (q xyzw, t)")
            abs_seq = torch.empty((max(K, 1), 7), dtype=torch.float64, device=self.device)
        ncorr = torch.empty(max(K, 1), dtype=torch.int32, device=self.device) if want_ncorr else None
        normal, valid, sx, si = table
        st = getattr(table, "strips", None) or (None, None)
        rc = _abi.lib().ssf_register_chain(
            self._h, _stream(self.device), K, _ptr(pb.xyzi), _ptr(pb.off), _ptr(pb.count),
            _ptr(normal), _ptr(valid), _ptr(sx), _ptr(si), int(pb.xyzi.shape[0]), pb.max_points,
            _ptr(pose_init), _ptr(seq), _ptr(pose_abs_init), _ptr(abs_seq), _ptr(ncorr),
            _ptr(st[0]), _ptr(st[1]))
        self._check(rc, "ssf_register_chain")
        return dict(pose_seq=seq[:K], pose_abs_seq=None if abs_seq is None else abs_seq[:K],
                    ncorr=None if ncorr is None else ncorr[:K])

    def register(self, last: PlaneBatch, last_table, curr: PlaneBatch, pose_rel, pose_abs=None,
                 want_log=False, want_nn=False, want_nlog=False, edges=None):
        """frameRegistration for P pairs (last[p], curr[p]).  pose_rel [P,7] f64 (q xyzw, t) is the
        warm start in and the solution out; pose_abs [P,7] is accumulated in place if given.
        edges = (last edges PlaneBatch, edge_table(last edges), curr edges PlaneBatch) adds the
        point-to-line blocks (beyond the reference, ssf_register_batch_edges)."""
        P = curr.count.numel()
        pose_rel = self._dev(pose_rel, torch.float64)
        if pose_abs is not None:
            pose_abs = self._dev(pose_abs, torch.float64)
        normal, valid, sx, si = last_table
        st = getattr(last_table, "strips", None) or (None, None)
        log = nlog = nn = None
        ncorr = torch.empty(P, dtype=torch.int32, device=self.device)
        if want_log:
            log = torch.zeros((P, self.cfg.max_iter, 10), dtype=torch.float64, device=self.device)
        if want_log or want_nlog:
            nlog = torch.zeros(P, dtype=torch.int32, device=self.device)
        if want_nn:
            nn = torch.full((curr.xyzi.shape[0],), -1, dtype=torch.int32, device=self.device)
        mx = max(last.max_points, curr.max_points)
        if edges is None:
            rc = _abi.lib().ssf_register_batch(
                self._h, _stream(self.device), P, _ptr(last.xyzi), _ptr(last.off), _ptr(last.count),
                _ptr(normal), _ptr(valid), _ptr(sx), _ptr(si), _ptr(curr.xyzi), _ptr(curr.off),
                _ptr(curr.count),
                int(curr.h_off[-1]), mx, _ptr(pose_rel), _ptr(pose_abs), _ptr(log), _ptr(nlog),
                _ptr(ncorr), _ptr(nn), _ptr(st[0]), _ptr(st[1]))
            self._check(rc, "ssf_register_batch")
            return dict(pose_rel=pose_rel, pose_abs=pose_abs, ncorr=ncorr, log=log, nlog=nlog, nn=nn)
        last_e, (line, lvalid), curr_e = edges
        if want_nn:
            raise ValueError("want_nn is not available with edges")
        ncorr_e = torch.empty(P, dtype=torch.int32, device=self.device)
        mxe = max(last_e.max_points, curr_e.max_points)
        rc = _abi.lib().ssf_register_batch_edges(
            self._h, _stream(self.device), P, _ptr(last.xyzi), _ptr(last.off), _ptr(last.count),
            _ptr(normal), _ptr(valid), _ptr(sx), _ptr(si), _ptr(curr.xyzi), _ptr(curr.off),
            _ptr(curr.count), int(curr.h_off[-1]), mx,
            _ptr(last_e.xyzi), _ptr(last_e.off), _ptr(last_e.count), _ptr(line), _ptr(lvalid),
            _ptr(curr_e.xyzi), _ptr(curr_e.off), _ptr(curr_e.count), int(curr_e.h_off[-1]), mxe,
            _ptr(pose_rel), _ptr(pose_abs), _ptr(log), _ptr(nlog), _ptr(ncorr), _ptr(ncorr_e),
            _ptr(st[0]), _ptr(st[1]))
        self._check(rc, "ssf_register_batch_edges")
        return dict(pose_rel=pose_rel, pose_abs=pose_abs, ncorr=ncorr, ncorr_edge=ncorr_e, log=log,
                    nlog=nlog, nn=None)

    # ------------------------------------------------------------------ PointCloudOdometry*.py
    def mask_pose(self, pts, flow, off, h_off, mode="gmm", mask_in=None, draws=None,
                  reflection=0, want_mask=True, out=None):
        """Mask + Kabsch for F frames -> (out [F,32] f64, bg_mask [total] u8 or None).
        pts / flow both float32 (ssf_mask_pose_batch) or both float64 (ssf_mask_pose_batch_f64:
        no rounding of f64 inputs).  out: optional preallocated (pose out [>= F, 32] f64,
        bg_mask [>= total] u8 or None)."""
        dt = torch.float64 if pts.dtype == torch.float64 else torch.float32
        pts = self._dev(pts, dt)
        flow = self._dev(flow, dt)
        F = h_off.numel() - 1
        total = int(h_off[-1])
        if out is not None:
            bg = (self._out(out[1], (max(total, 1),), torch.uint8, "bg_mask out")
                  if want_mask and out[1] is not None else None)
            out = self._out(out[0], (max(F, 1), _abi.POSE_OUT_STRIDE), torch.float64, "pose out")
            if want_mask and bg is None:
                raise ValueError("want_mask needs a bg_mask out buffer")
        else:
            out = torch.empty((max(F, 1), _abi.POSE_OUT_STRIDE), dtype=torch.float64, device=self.device)
            bg = torch.empty(max(total, 1), dtype=torch.uint8, device=self.device) if want_mask else None
        h_off64 = h_off.to(torch.int64).contiguous()
        hd = None
        if draws is not None:
            hd = torch.as_tensor(draws, dtype=torch.float64).reshape(-1).contiguous()
            if hd.numel() != 3 * F:
                raise SSFError("draws must hold 3 doubles per frame")
        if mask_in is not None:
            mask_in = self._dev(mask_in, torch.uint8)
        name = "ssf_mask_pose_batch_f64" if dt == torch.float64 else "ssf_mask_pose_batch"
        rc = getattr(_abi.lib(), name)(
            self._h, _stream(self.device), F, _ptr(pts), _ptr(flow), _ptr(off),
            C.c_void_p(h_off64.data_ptr()), MASK_MODES[mode], _ptr(mask_in),
            None if hd is None else C.c_void_p(hd.data_ptr()), int(reflection), _ptr(bg), _ptr(out))
        self._check(rc, name)
        return out[:F], (bg[:total] if bg is not None else None)

    def kabsch_f32(self, dst, off, h_off, src=None, flow=None, mask=None, reflection=0, out=None):
        """slove_RT_by_SVD + Quaternion on float32 arrays per frame (ssf_kabsch_f32_batch, the ASF
        block's arithmetic, main_sju_occ_ros.py:273-284): source rows dst + flow (f32) or src;
        rows with mask != 0.  out: mask_pose()'s output for the same frames (its fit fields are
        kept, T / Q / R / NBG / STATUS replaced in place), or None for a fresh [F, 32] tensor."""
        dst = self._dev(dst, torch.float32)
        src = None if src is None else self._dev(src, torch.float32)
        flow = None if flow is None else self._dev(flow, torch.float32)
        if (src is None) == (flow is None):
            raise SSFError("kabsch_f32: give exactly one of src / flow")
        mask = None if mask is None else self._dev(mask, torch.uint8)
        off = self._dev(off, torch.int64)
        F = h_off.numel() - 1
        if off.numel() != F + 1:
            raise ValueError(f"off has {off.numel()} entries for {F} frames")
        total = int(h_off[-1])
        for name, t, per in (("dst", dst, 3), ("src", src, 3), ("flow", flow, 3), ("mask", mask, 1)):
            if t is not None and t.numel() != per * total:
                raise ValueError(f"{name} has {t.numel()} values for {total} points ({per} per point)")
        after = out is not None
        if out is None:
            out = torch.empty((max(F, 1), _abi.POSE_OUT_STRIDE), dtype=torch.float64, device=self.device)
        else:
            out = self._dev(out, torch.float64)
            if out.dim() != 2 or out.shape[0] < F or out.shape[1] != _abi.POSE_OUT_STRIDE:
                raise ValueError(f"out must be [>= {F}, {_abi.POSE_OUT_STRIDE}] float64, got {tuple(out.shape)}")
        rc = _abi.lib().ssf_kabsch_f32_batch(self._h, _stream(self.device), F, _ptr(src), _ptr(dst),
                                             _ptr(flow), _ptr(off), _ptr(mask), int(reflection),
                                             1 if after else 0, _ptr(out))
        self._check(rc, "ssf_kabsch_f32_batch")
        return out[:F]

    def accumulate_sequence(self, rel, start=None):
        rel = self._dev(rel, torch.float64)
        n = rel.shape[0]
        out = torch.empty_like(rel)
        hs = None if start is None else torch.as_tensor(start, dtype=torch.float64).contiguous()
        rc = _abi.lib().ssf_accumulate_sequence(self._h, _stream(self.device), n, _ptr(rel),
                                                None if hs is None else C.c_void_p(hs.data_ptr()),
                                                _ptr(out))
        self._check(rc, "ssf_accumulate_sequence")
        return out


def identity_poses(n, device):
    p = torch.zeros((n, 7), dtype=torch.float64, device=device)
    p[:, 3] = 1.0
    return p

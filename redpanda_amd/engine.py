"""Host-side segment engine over the C-ABI.

`Engine` owns one rpgpu context (one per host thread / shard, as the
reference's shard-per-core ownership requires: SURVEY.md §8(b)).  Device
buffers are torch tensors — torch is plumbing here (HIP allocation, streams,
torch.distributed for the final gather); all compute is in librpgpu.so.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import abi
from ._lib import CapacityC, JobC, RpgpuError, check, load


def _torch():
    import torch
    return torch


@dataclass
class DeviceResult:
    batches: "object"     # torch uint8 tensor viewed as abi.BATCH_RESULT on the host
    records: "object"
    decoded: "object"
    summaries: "object"
    totals: "object"
    bitmap: "object"
    n_segments: int

    def totals_host(self):
        return np.frombuffer(self.totals.cpu().numpy().tobytes(), dtype=abi.JOB_TOTALS)[0]

    def to_host(self):
        t = self.totals_host()
        nb = int(min(t["n_batches"], self.batches.numel() // abi.BATCH_RESULT.itemsize))
        nr = int(min(t["n_records"], self.records.numel() // abi.RECORD_INDEX.itemsize))
        nd = int(min(t["decoded_bytes"], self.decoded.numel()))
        b = np.frombuffer(self.batches[: nb * abi.BATCH_RESULT.itemsize].cpu().numpy().tobytes(), dtype=abi.BATCH_RESULT)
        r = np.frombuffer(self.records[: nr * abi.RECORD_INDEX.itemsize].cpu().numpy().tobytes(), dtype=abi.RECORD_INDEX)
        d = self.decoded[:nd].cpu().numpy()
        s = np.frombuffer(self.summaries.cpu().numpy().tobytes(), dtype=abi.SEGMENT_SUMMARY)[: self.n_segments]
        bm = self.bitmap[: (nb + 63) // 64 * 8].cpu().numpy().view(np.uint64) if self.bitmap is not None else None
        return HostResult(b, r, d, s, t, bm)


@dataclass
class HostResult:
    batches: np.ndarray
    records: np.ndarray
    decoded: np.ndarray
    summaries: np.ndarray
    totals: np.void
    bitmap: np.ndarray


class Engine:
    """One rpgpu context on one device."""

    def __init__(self, device: int = 0):
        torch = _torch()
        if not torch.cuda.is_available():
            raise RpgpuError("no GPU visible: the engine has no CPU fallback")
        self.L = load()
        self.device = device
        torch.cuda.set_device(device)
        ctx = C.c_void_p()
        check(self.L.rpgpu_create(device, C.byref(ctx)), None, "rpgpu_create")
        self.ctx = ctx

    def close(self):
        if getattr(self, "ctx", None):
            self.L.rpgpu_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self, dev, stream):
        """The stream to launch on, and a finish() that orders torch's current
        stream after the launch.  torch's legacy default stream (handle 0)
        would make the library fall back to its private non-blocking stream,
        which torch neither waits on nor tracks; such launches go to a torch
        side stream that waits on the current one first."""
        torch = _torch()
        cur = torch.cuda.current_stream(dev)
        s = stream if stream is not None else cur
        if s.cuda_stream != 0:
            return s, lambda *tensors: None
        side = getattr(self, "_side", None)
        if side is None or side.device != dev:
            side = self._side = torch.cuda.Stream(dev)
        side.wait_stream(s)

        def finish(*tensors):
            s.wait_stream(side)
            for t in tensors:
                if t is not None:
                    t.record_stream(side)
        return side, finish

    def set_timing(self, on: bool = True):
        check(self.L.rpgpu_set_timing(self.ctx, 1 if on else 0), self.ctx, "rpgpu_set_timing")

    def last_timings(self):
        ms = (C.c_float * 6)()
        check(self.L.rpgpu_last_timings(self.ctx, ms, 6), self.ctx, "rpgpu_last_timings")
        return {"total": ms[0], "discover": ms[1], "resolve_plan": ms[2], "validate": ms[3], "decode": ms[4],
                "walk": ms[5]}

    def alloc_outputs(self, n_segments: int, batch_capacity: int, record_capacity: int,
                      decoded_capacity: int, bitmap: bool = True):
        torch = _torch()
        dev = torch.device("cuda", self.device)
        u8 = torch.uint8
        return DeviceResult(
            batches=torch.zeros(max(batch_capacity, 1) * abi.BATCH_RESULT.itemsize, dtype=u8, device=dev),
            records=torch.zeros(max(record_capacity, 1) * abi.RECORD_INDEX.itemsize, dtype=u8, device=dev),
            decoded=torch.zeros(max(decoded_capacity, 1), dtype=u8, device=dev),
            summaries=torch.zeros(max(n_segments, 1) * abi.SEGMENT_SUMMARY.itemsize, dtype=u8, device=dev),
            totals=torch.zeros(abi.JOB_TOTALS.itemsize, dtype=u8, device=dev),
            bitmap=torch.zeros(((max(batch_capacity, 1) + 63) // 64) * 8, dtype=u8, device=dev) if bitmap else None,
            n_segments=n_segments,
        )

    def _job(self, data, seg_offsets, out, flags, chunk_bytes, d_seg_offsets, layout):
        torch = _torch()
        h_off = np.ascontiguousarray(np.asarray(seg_offsets, dtype=np.uint64))
        if d_seg_offsets is None:
            d_seg_offsets = torch.from_numpy(h_off.view(np.int64)).to(data.device)
        job = JobC()
        job.d_data = data.data_ptr()
        job.d_seg_offsets = d_seg_offsets.data_ptr()
        job.h_seg_offsets = h_off.ctypes.data
        job.n_segments = h_off.size - 1
        job.layout = layout
        job.flags = flags
        job.chunk_bytes = chunk_bytes
        if out is not None:
            job.d_batches = out.batches.data_ptr()
            job.batch_capacity = out.batches.numel() // abi.BATCH_RESULT.itemsize
            job.d_records = out.records.data_ptr()
            job.record_capacity = out.records.numel() // abi.RECORD_INDEX.itemsize
            job.d_decoded = out.decoded.data_ptr()
            job.decoded_capacity = out.decoded.numel()
            job.d_summaries = out.summaries.data_ptr()
            job.d_totals = out.totals.data_ptr()
            job.d_valid_bitmap = out.bitmap.data_ptr() if out.bitmap is not None else 0
        return job, (h_off, d_seg_offsets)

    def query_capacity(self, data, seg_offsets, flags: int = abi.JOB_CRC | abi.JOB_PARSE, chunk_bytes: int = 0,
                       layout: int = abi.LAYOUT_DISK, stream=None):
        """rpgpu_query_capacity: (n_batches, record_capacity, decoded_capacity)
        the job needs, before it runs (synchronous)."""
        job, keep = self._job(data, seg_offsets, None, flags, chunk_bytes, None, layout)
        s, finish = self._stream(data.device, stream)
        cap = CapacityC()
        check(self.L.rpgpu_query_capacity(self.ctx, C.byref(job), C.c_void_p(s.cuda_stream), C.byref(cap)), self.ctx,
              "rpgpu_query_capacity")
        finish(data, keep[1])
        return int(cap.n_batches), int(cap.record_capacity), int(cap.decoded_capacity)

    def submit_async(self, data, seg_offsets, out: DeviceResult, flags: int = abi.JOB_CRC | abi.JOB_PARSE,
                     chunk_bytes: int = 0, layout: int = abi.LAYOUT_DISK):
        """rpgpu_submit_async on the context's own stream: returns a Pending
        whose poll() never blocks.  Inputs and outputs stay referenced by it
        until it completes."""
        job, keep = self._job(data, seg_offsets, out, flags, chunk_bytes, None, layout)
        torch = _torch()
        torch.cuda.current_stream(data.device).synchronize()  # inputs written by torch are complete
        p = C.c_void_p()
        check(self.L.rpgpu_submit_async(self.ctx, C.byref(job), None, C.byref(p)), self.ctx, "rpgpu_submit_async")
        return Pending(self, p, (data, out, keep))

    def uncompress_batch(self, codecs, payloads, caps=None):
        """rpgpu_uncompress_batch: [(status, bytes)] per payload, one device
        round trip for the lz4/snappy ones."""
        n = len(payloads)
        srcs = [np.frombuffer(bytes(p), dtype=np.uint8) for p in payloads]
        caps = caps or [max(len(p) * 300, 1 << 20) for p in payloads]
        outs = [np.zeros(max(c, 1), dtype=np.uint8) for c in caps]
        ci = (C.c_int * max(n, 1))(*codecs)
        ip = (C.c_void_p * max(n, 1))(*[s.ctypes.data for s in srcs])
        il = (C.c_size_t * max(n, 1))(*[s.nbytes for s in srcs])
        op = (C.c_void_p * max(n, 1))(*[o.ctypes.data for o in outs])
        oc = (C.c_size_t * max(n, 1))(*caps)
        ol = (C.c_size_t * max(n, 1))()
        st = (C.c_int * max(n, 1))()
        check(self.L.rpgpu_uncompress_batch(self.ctx, n, ci, ip, il, op, oc, ol, st), self.ctx, "rpgpu_uncompress_batch")
        return [(int(st[i]), outs[i][: ol[i]].tobytes() if st[i] == 0 else int(ol[i])) for i in range(n)]

    def compress_batch(self, codecs, payloads, frags=None, caps=None):
        """rpgpu_compress_batch (compressor::compress on the device): [(status,
        bytes)] per payload — lz4 frames / snappy-java streams (frags[i]: the
        iobuf fragment size, 0 = one fragment)."""
        n = len(payloads)
        srcs = [np.frombuffer(bytes(p), dtype=np.uint8) if len(p) else np.zeros(1, np.uint8) for p in payloads]
        frags = list(frags) if frags is not None else [0] * n
        caps = caps or [max(int(self.L.rpgpu_compress_bound(c, len(p), f)), 1) for c, p, f in zip(codecs, payloads, frags)]
        outs = [np.zeros(max(c, 1), dtype=np.uint8) for c in caps]
        ci = (C.c_int * max(n, 1))(*codecs)
        ip = (C.c_void_p * max(n, 1))(*[s.ctypes.data for s in srcs])
        il = (C.c_size_t * max(n, 1))(*[len(p) for p in payloads])
        fr = (C.c_size_t * max(n, 1))(*frags)
        op = (C.c_void_p * max(n, 1))(*[o.ctypes.data for o in outs])
        oc = (C.c_size_t * max(n, 1))(*caps)
        ol = (C.c_size_t * max(n, 1))()
        st = (C.c_int * max(n, 1))()
        check(self.L.rpgpu_compress_batch(self.ctx, n, ci, ip, il, fr, op, oc, ol, st), self.ctx, "rpgpu_compress_batch")
        return [(int(st[i]), outs[i][: ol[i]].tobytes() if st[i] == 0 else int(ol[i])) for i in range(n)]

    def stamp(self, data, positions, payload_lens, next_offset: int = 0,
              flags: int = abi.STAMP_OFFSETS | abi.STAMP_CRC, stream=None):
        """rpgpu_stamp: stamp the headers of disk-layout batches in `data` (a
        torch uint8 CUDA tensor with 16 readable bytes past the last payload)
        in place — appender offsets from next_offset, size/crc
        (reset_size_checksum_metadata) and header_crc."""
        torch = _torch()
        dev = data.device
        pos = torch.from_numpy(np.ascontiguousarray(np.asarray(positions, dtype=np.uint64)).view(np.int64)).to(dev)
        pl = torch.from_numpy(np.ascontiguousarray(np.asarray(payload_lens, dtype=np.uint32)).view(np.int32)).to(dev)
        s, finish = self._stream(dev, stream)
        check(self.L.rpgpu_stamp(self.ctx, C.c_void_p(data.data_ptr()), C.c_void_p(pos.data_ptr()),
                                 C.c_void_p(pl.data_ptr()), int(pos.numel()), int(next_offset), int(flags),
                                 C.c_void_p(s.cuda_stream)), self.ctx, "rpgpu_stamp")
        finish(data, pos, pl)
        return data

    @staticmethod
    def seed_tensors(seeds, device):
        """Per-segment ascending batch positions (e.g. an index's position
        entries) -> (d_seeds, d_seed_offsets) for the index-seeded mode."""
        torch = _torch()
        arrs = [np.asarray(x, dtype=np.uint64).ravel() for x in seeds]
        offs = np.cumsum([0] + [a.size for a in arrs]).astype(np.uint64)
        flat = np.concatenate(arrs) if arrs and offs[-1] else np.zeros(1, dtype=np.uint64)
        return (torch.from_numpy(flat.view(np.int64).copy()).to(device),
                torch.from_numpy(offs.view(np.int64).copy()).to(device))

    def serialize_wire(self, data, seg_offsets, out: DeviceResult, first: int = 0, n: int = None, stream=None):
        """rpgpu_serialize_wire: batches [first, first + n) of a completed
        disk-layout job as a Kafka v2 record set (device uint8 tensor)."""
        torch = _torch()
        dev = data.device
        if n is None:
            n = int(out.totals_host()["n_batches"]) - first
        sizes = np.frombuffer(out.batches[first * abi.BATCH_RESULT.itemsize:(first + n) * abi.BATCH_RESULT.itemsize]
                              .cpu().numpy().tobytes(), dtype=abi.BATCH_RESULT)["size_bytes"]
        cap = int(np.sum(sizes.astype(np.int64))) + 16
        wire = torch.empty(max(cap, 16), dtype=torch.uint8, device=dev)
        total = torch.zeros(1, dtype=torch.int64, device=dev)
        d_off = torch.from_numpy(np.ascontiguousarray(np.asarray(seg_offsets, dtype=np.uint64)).view(np.int64)).to(dev)
        s, finish = self._stream(dev, stream)
        check(self.L.rpgpu_serialize_wire(self.ctx, C.c_void_p(data.data_ptr()), C.c_void_p(d_off.data_ptr()),
                                          C.c_void_p(out.batches.data_ptr()), int(first), int(n),
                                          C.c_void_p(wire.data_ptr()), C.c_void_p(total.data_ptr()),
                                          C.c_void_p(s.cuda_stream)), self.ctx, "rpgpu_serialize_wire")
        finish(data, d_off, out.batches, wire, total)
        s.synchronize()
        return wire[: int(total.item())]

    def submit(self, data, seg_offsets, out: DeviceResult, flags: int = abi.JOB_CRC | abi.JOB_PARSE,
               chunk_bytes: int = 0, stream=None, d_seg_offsets=None, layout: int = abi.LAYOUT_DISK, seeds=None):
        """Enqueue one job ordered on `stream` (default: torch's current
        stream; the launch itself goes to a side stream when that is the
        legacy default stream, see _stream).  `data` is a torch uint8 CUDA
        tensor holding the concatenated segments (abi.LAYOUT_DISK: Redpanda
        log segments; abi.LAYOUT_WIRE: Kafka v2 record sets as a produce
        request carries them).  Inputs and outputs are kept alive for the
        allocator until the job is done."""
        torch = _torch()
        h_off = np.ascontiguousarray(np.asarray(seg_offsets, dtype=np.uint64))
        if d_seg_offsets is None:
            d_seg_offsets = torch.from_numpy(h_off.view(np.int64)).to(data.device)
        self._keep = (h_off, d_seg_offsets)
        job = JobC()
        job.d_data = data.data_ptr()
        job.d_seg_offsets = d_seg_offsets.data_ptr()
        job.h_seg_offsets = h_off.ctypes.data
        job.n_segments = h_off.size - 1
        job.layout = layout
        job.flags = flags
        job.chunk_bytes = chunk_bytes
        job.d_batches = out.batches.data_ptr()
        job.batch_capacity = out.batches.numel() // abi.BATCH_RESULT.itemsize
        job.d_records = out.records.data_ptr()
        job.record_capacity = out.records.numel() // abi.RECORD_INDEX.itemsize
        job.d_decoded = out.decoded.data_ptr()
        job.decoded_capacity = out.decoded.numel()
        job.d_summaries = out.summaries.data_ptr()
        job.d_totals = out.totals.data_ptr()
        job.d_valid_bitmap = out.bitmap.data_ptr() if out.bitmap is not None else 0
        sd = so = None
        if seeds is not None:
            sd, so = seeds if isinstance(seeds, tuple) else self.seed_tensors(seeds, data.device)
            job.d_seeds, job.d_seed_offsets = sd.data_ptr(), so.data_ptr()
            self._keep_seeds = (sd, so)  # alive until the next submit
        s, finish = self._stream(data.device, stream)
        check(self.L.rpgpu_submit(self.ctx, C.byref(job), C.c_void_p(s.cuda_stream)), self.ctx, "rpgpu_submit")
        finish(data, d_seg_offsets, out.batches, out.records, out.decoded, out.summaries, out.totals, out.bitmap, sd, so)
        return out

    def segment_index(self, out: DeviceResult, base_offsets, step: int = abi.INDEX_DEFAULT_STEP, stream=None,
                      outputs=None):
        """Rebuild each segment's sparse index (segment_index::maybe_track over
        the crc-good prefix, storage/log_replayer.cc:62-74) from a completed
        disk-layout job `out`, on the device.  Returns device tensors
        (states, relative_offset, relative_time, position); segment s's
        entries are [first_entry, first_entry + n_entries) of each array.
        `outputs` reuses a previous call's returned tensors (same job shape)."""
        torch = _torch()
        dev = out.batches.device
        nseg = out.n_segments
        cap = out.batches.numel() // abi.BATCH_RESULT.itemsize
        if outputs is None:
            st = np.zeros(max(nseg, 1), dtype=abi.INDEX_STATE)
            st["base_offset"][:nseg] = np.asarray(base_offsets, dtype=np.int64)
            states = torch.from_numpy(st.view(np.uint8).copy()).to(dev)
            rel_off = torch.zeros(max(cap, 1), dtype=torch.int32, device=dev)
            rel_time = torch.zeros(max(cap, 1), dtype=torch.int32, device=dev)
            pos = torch.zeros(max(cap, 1), dtype=torch.int64, device=dev)
        else:
            # base_offset is an input the kernels keep; every other field is rewritten
            states, rel_off, rel_time, pos = outputs
            if states.numel() < nseg * abi.INDEX_STATE.itemsize or min(rel_off.numel(), rel_time.numel(),
                                                                       pos.numel()) < cap:
                raise RpgpuError("segment_index: `outputs` smaller than this job's segments / batch capacity")
            have = np.frombuffer(states[: nseg * abi.INDEX_STATE.itemsize].cpu().numpy().tobytes(),
                                 dtype=abi.INDEX_STATE)["base_offset"]
            if not np.array_equal(have, np.asarray(base_offsets, dtype=np.int64)[:nseg]):
                raise RpgpuError("segment_index: `outputs` were built for other base offsets")
        s, finish = self._stream(dev, stream)
        check(self.L.rpgpu_segment_index(self.ctx, C.c_void_p(out.batches.data_ptr()), cap,
                                         C.c_void_p(out.summaries.data_ptr()), nseg, step,
                                         C.c_void_p(states.data_ptr()), C.c_void_p(rel_off.data_ptr()),
                                         C.c_void_p(rel_time.data_ptr()), C.c_void_p(pos.data_ptr()),
                                         C.c_void_p(s.cuda_stream)), self.ctx, "rpgpu_segment_index")
        finish(out.batches, out.summaries, states, rel_off, rel_time, pos)
        return states, rel_off, rel_time, pos

    @staticmethod
    def index_to_host(states, rel_off, rel_time, pos, n_segments: int):
        """Per segment: (index_state row, relative_offset, relative_time, position) numpy."""
        _torch().cuda.synchronize(states.device)
        st = np.frombuffer(states.cpu().numpy().tobytes(), dtype=abi.INDEX_STATE)[:n_segments]
        ro = rel_off.cpu().numpy().view(np.uint32)
        rt = rel_time.cpu().numpy().view(np.uint32)
        ps = pos.cpu().numpy().view(np.uint64)
        out = []
        for s in st:
            a, n = int(s["first_entry"]), int(s["n_entries"])
            out.append((s, ro[a:a + n].copy(), rt[a:a + n].copy(), ps[a:a + n].copy()))
        return out

    def uncompress(self, codec: int, payload: bytes, cap: int = None):
        """compression::compressor::uncompress for one payload on the device.
        Returns the decoded bytes; raises RpgpuError (RPGPU_E_CODEC) where the
        reference throws std::runtime_error."""
        src = np.frombuffer(bytes(payload), dtype=np.uint8)
        if cap is None:
            cap = max(len(payload) * 300, 1 << 20)
        out = np.zeros(max(cap, 1), dtype=np.uint8)
        n = C.c_size_t(0)
        rc = self.L.rpgpu_uncompress(self.ctx, codec, src.ctypes.data_as(C.c_void_p), src.nbytes,
                                     out.ctypes.data_as(C.c_void_p), cap, C.byref(n))
        check(rc, self.ctx, "rpgpu_uncompress")
        return out[: n.value].tobytes()

    def validate(self, data, seg_offsets, flags: int = abi.JOB_CRC | abi.JOB_PARSE, batch_capacity=None,
                 record_capacity=None, decoded_capacity=None, chunk_bytes: int = 0,
                 layout: int = abi.LAYOUT_DISK, seeds=None) -> HostResult:
        """Convenience: allocate outputs, run, synchronize, copy back."""
        torch = _torch()
        offs = np.asarray(seg_offsets, dtype=np.uint64)
        total = int(offs[-1])
        nseg = offs.size - 1
        if batch_capacity is None:
            batch_capacity = total // abi.HEADER_SIZE + nseg + 1
        if record_capacity is None:
            record_capacity = max(total // 4, 64)
        if decoded_capacity is None:
            decoded_capacity = max(total * 8, 1 << 16) if flags & abi.JOB_DECODE else 1
        out = self.alloc_outputs(nseg, batch_capacity, record_capacity, decoded_capacity)
        self.submit(data, offs, out, flags, chunk_bytes, layout=layout, seeds=seeds)
        torch.cuda.synchronize(data.device)
        return out.to_host()

    def validate_host(self, segments, flags: int = abi.JOB_CRC | abi.JOB_PARSE, layout: int = abi.LAYOUT_DISK,
                      batch_capacity=None, group_kib: int = 0, record_capacity=None, decoded_capacity=None,
                      index_step: int = 0, base_offsets=None):
        """rpgpu_validate_host: host-resident segments (numpy uint8 arrays,
        pinned or pageable) copied to the device in double-buffered groups
        and validated there.  Returns a HostResult (batches, records, decoded
        arena, summaries, totals; bitmap None) holding what one device job
        over all the segments returns, plus `.index` (per segment:
        index_state row, relative_offset, relative_time, position) when
        index_step is set."""
        segs = [np.ascontiguousarray(s, dtype=np.uint8) for s in segments]
        n = len(segs)
        total = sum(s.size for s in segs)
        if batch_capacity is None:
            batch_capacity = total // abi.HEADER_SIZE + n + 1
        if record_capacity is None:
            record_capacity = max(total // 4, 64) if flags & abi.JOB_PARSE else 0
        if decoded_capacity is None:
            decoded_capacity = max(total * 8, 1 << 16) if flags & abi.JOB_DECODE else 0
        ptrs = (C.c_void_p * max(n, 1))(*[s.ctypes.data for s in segs])
        sizes = (C.c_uint64 * max(n, 1))(*[s.size for s in segs])
        batches = np.zeros(max(batch_capacity, 1), dtype=abi.BATCH_RESULT)
        recs = np.zeros(max(record_capacity, 1), dtype=abi.RECORD_INDEX)
        dec = np.zeros(max(decoded_capacity, 1), dtype=np.uint8)
        sums = np.zeros(max(n, 1), dtype=abi.SEGMENT_SUMMARY)
        tot = np.zeros(1, dtype=abi.JOB_TOTALS)
        st = np.zeros(max(n, 1), dtype=abi.INDEX_STATE)
        if base_offsets is not None:
            st["base_offset"][:n] = np.asarray(base_offsets, dtype=np.int64)
        ro = np.zeros(max(batch_capacity, 1), np.uint32)
        rt = np.zeros(max(batch_capacity, 1), np.uint32)
        ps = np.zeros(max(batch_capacity, 1), np.uint64)
        job = HostJobC(C.cast(ptrs, C.c_void_p), C.cast(sizes, C.c_void_p), n, layout, flags, group_kib,
                       batches.ctypes.data, batch_capacity, sums.ctypes.data, tot.ctypes.data,
                       recs.ctypes.data if record_capacity else None, record_capacity,
                       dec.ctypes.data if decoded_capacity else None, decoded_capacity,
                       index_step, st.ctypes.data if index_step else None, ro.ctypes.data if index_step else None,
                       rt.ctypes.data if index_step else None, ps.ctypes.data if index_step else None)
        rc = self.L.rpgpu_validate_host(self.ctx, C.byref(job))
        check(rc, self.ctx, "rpgpu_validate_host")
        t = tot[0]
        nb = int(min(t["n_batches"], batch_capacity))
        nr = int(min(t["n_records"], record_capacity))
        nd = int(min(t["decoded_bytes"], decoded_capacity))
        res = HostResult(batches[:nb], recs[:nr], dec[:nd], sums[:n], t, None)
        res.index = None
        if index_step:
            res.index = []
            for k in range(n):
                a, m = int(st[k]["first_entry"]), int(st[k]["n_entries"])
                res.index.append((st[k], ro[a:a + m].copy(), rt[a:a + m].copy(), ps[a:a + m].copy()))
        return res


class Pending:
    """An in-flight job (rpgpu_pending)."""

    def __init__(self, eng, handle, keep):
        self.eng, self.h, self._keep = eng, handle, keep

    def poll(self) -> bool:
        rc = self.eng.L.rpgpu_poll(self.h)
        if rc == abi.PENDING:
            return False
        check(rc, self.eng.ctx, "rpgpu_poll")
        return True

    def wait(self):
        check(self.eng.L.rpgpu_wait(self.h), self.eng.ctx, "rpgpu_wait")

    def release(self):
        if self.h:
            self.eng.L.rpgpu_release(self.h)
            self.h = None
            self._keep = None

    def __del__(self):
        try:
            if self.h:
                self.wait()
            self.release()
        except Exception:
            pass


class HostJobC(C.Structure):
    """rpgpu_host_job (include/rpgpu.h)."""
    _fields_ = [("segments", C.c_void_p), ("seg_sizes", C.c_void_p), ("n_segments", C.c_uint32),
                ("layout", C.c_uint32), ("flags", C.c_uint32), ("group_kib", C.c_uint32),
                ("batches", C.c_void_p), ("batch_capacity", C.c_uint64), ("summaries", C.c_void_p),
                ("totals", C.c_void_p), ("records", C.c_void_p), ("record_capacity", C.c_uint64),
                ("decoded", C.c_void_p), ("decoded_capacity", C.c_uint64), ("index_step", C.c_uint64),
                ("index_states", C.c_void_p), ("rel_offset", C.c_void_p), ("rel_time", C.c_void_p),
                ("position", C.c_void_p)]

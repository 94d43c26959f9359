"""A/B timing of kernel variants in ONE process (interleaved rounds), for tuning.

    python scripts/microbench.py [--segments 32] [--rounds 5]
Prints one JSON line per variant: median/min GB/s of frame bytes over the rounds."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segments", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="crc,framing,commit,lease", help="comma list of sections to run")
    ap.add_argument("--ablation", action="store_true", help="also time the CRC access-pattern ablation")
    a = ap.parse_args()
    import torch

    from ratis_amd import _lib, engine, workload
    ctx = engine.Context(0)
    # calibration: what plain torch streaming kernels reach on this device
    x = torch.empty(1 << 27, dtype=torch.int64, device="cuda").random_()
    y = torch.empty_like(x)
    for name, fn, nbytes in (("copy_1GiB", lambda: y.copy_(x), 2 * x.numel() * 8),
                             ("sum_1GiB", lambda: x.sum(), x.numel() * 8)):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"kernel": "calibration:" + name, "GBps": round(nbytes / (e0.elapsed_time(e1) / 10 * 1e-3) / 1e9, 1)}))
    del x, y
    ss = workload.synth_segments(ctx, n_segments=a.segments, corrupt_rate=0)
    fb = ss.batch
    only = set(a.only.split(","))
    nv = engine.crc32c_num_variants() if "crc" in only else 0
    if "crc" in only and a.ablation:
        # access-pattern ablation (variant nv): v8's loads and stores, no table fold
        for r in range(a.rounds):
            engine.crc32c_frames(ctx, fb, flags=0, variant=nv)   # no verify: its CRCs are not exact
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                engine.crc32c_frames(ctx, fb, flags=0, variant=nv)
            e1.record()
            torch.cuda.synchronize()
            print(json.dumps({"kernel": "crc32c_ablation_loads_only", "variant": nv,
                              "GBps": round(ss.frame_bytes / (e0.elapsed_time(e1) / a.iters * 1e-3) / 1e9, 1)}), flush=True)
            # the same kernel, exact variant 24, also without verify (same comparison basis)
            engine.crc32c_frames(ctx, fb, flags=0, variant=24)
            e0.record()
            for _ in range(a.iters):
                engine.crc32c_frames(ctx, fb, flags=0, variant=24)
            e1.record()
            torch.cuda.synchronize()
            print(json.dumps({"kernel": "crc32c_no_verify", "variant": 24,
                              "GBps": round(ss.frame_bytes / (e0.elapsed_time(e1) / a.iters * 1e-3) / 1e9, 1)}), flush=True)
    res = {v: [] for v in range(nv)}
    for r in range(a.rounds):
        for v in range(nv):
            engine.crc32c_frames(ctx, fb, flags=_lib.RH_CRC_VERIFY, variant=v)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                engine.crc32c_frames(ctx, fb, flags=_lib.RH_CRC_VERIFY, variant=v)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            res[v].append(ss.frame_bytes / (ms * 1e-3) / 1e9)
            assert int(fb.n_bad.item()) == 0
    for v in range(nv):
        x = np.array(res[v])
        print(json.dumps({"kernel": "crc32c", "variant": v, "median_GBps": round(float(np.median(x)), 1),
                          "min_GBps": round(float(x.min()), 1), "max_GBps": round(float(x.max()), 1)}))
    # segment framing walk: variants x segment shapes (same 8 GiB footprint)
    del fb
    lib = _lib.load()

    def framing(ss, tag):
        n = ss.n_segments
        sb = engine.SegmentBatch(buf=ss.batch.buf,
                                 seg_off=torch.arange(n, device="cuda", dtype=torch.int64) * ss.segment_size,
                                 seg_len=torch.full((n,), ss.segment_size, device="cuda", dtype=torch.int64),
                                 frames_per_seg_cap=ss.frames_per_segment + 16)
        for v in range(6):
            _lib.check(lib.rh_segments_set_variant(v))
            fr = []
            for r in range(a.rounds):
                engine.segments_scan(ctx, sb)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    engine.segments_scan(ctx, sb)
                e1.record()
                torch.cuda.synchronize()
                fr.append(n * ss.segment_size / (e0.elapsed_time(e1) / a.iters * 1e-3) / 1e9)
                assert int(sb.total_frames.item()) == n * ss.frames_per_segment
            x = np.array(fr)
            print(json.dumps({"kernel": "segments_scan", "variant": v, "shape": tag, "segments": n,
                              "median_GBps": round(float(np.median(x)), 1), "min_GBps": round(float(x.min()), 1),
                              "max_GBps": round(float(x.max()), 1)}), flush=True)
        _lib.check(lib.rh_segments_set_variant(1))

    if "framing" not in only:
        ss = None
    else:
        framing(ss, "32MiBx4KiB")
        total = ss.n_segments * ss.segment_size
        del ss
        torch.cuda.empty_cache()
        ss = workload.synth_segments(ctx, n_segments=total // (4 << 20), segment_size=4 << 20, corrupt_rate=0)
        framing(ss, "4MiBx4KiB")
        del ss
        torch.cuda.empty_cache()
        ss = workload.synth_segments(ctx, n_segments=a.segments, frame_size=512, corrupt_rate=0)
        framing(ss, "32MiBx512B")
        del ss
        torch.cuda.empty_cache()
        for lo, hi in ((64, 2048), (64, 512)):
            rs = workload.synth_ragged_segments(ctx, n_segments=a.segments, min_frame=lo, max_frame=hi)
            n = rs.n_segments
            sb = engine.SegmentBatch(buf=rs.batch.buf,
                                     seg_off=torch.arange(n, device="cuda", dtype=torch.int64) * rs.segment_size,
                                     seg_len=torch.full((n,), rs.segment_size, device="cuda", dtype=torch.int64),
                                     frames_per_seg_cap=int(rs.seg_nframes.max()) + 16)
            for v in range(6):
                _lib.check(lib.rh_segments_set_variant(v))
                fr = []
                for r in range(a.rounds):
                    engine.segments_scan(ctx, sb)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.iters):
                        engine.segments_scan(ctx, sb)
                    e1.record()
                    torch.cuda.synchronize()
                    fr.append(n * rs.segment_size / (e0.elapsed_time(e1) / a.iters * 1e-3) / 1e9)
                    assert int(sb.total_frames.item()) == int(rs.seg_nframes.sum())
                    assert torch.equal(sb.frame_off[: rs.batch.frame_off.numel()], rs.batch.frame_off)
                x = np.array(fr)
                print(json.dumps({"kernel": "segments_scan", "variant": v, "shape": f"32MiBx{lo}-{hi}B ragged", "segments": n,
                                  "median_GBps": round(float(np.median(x)), 1)}), flush=True)
            _lib.check(lib.rh_segments_set_variant(1))
            ss = rs
    del ss
    # commit kernel variants over 8 rotating 1M-group batches (config 3)
    host = workload.commit_snapshot(1_000_000)
    alg = sum(h.algorithmic_bytes() for h in host)
    batches = []
    for r in range(8):
        tiers = []
        for h in host:
            t = workload.to_device(h)
            t.follower_index += r << 44
            t.self_index += r << 44
            t.commit_in += r << 44
            t.term_start += r << 44
            tiers.append(t.alloc_outputs())
        batches.append(tiers)
    lib = _lib.load()
    ncv = lib.rh_commit_num_variants() if "commit" in only else 0
    cres = {v: [] for v in range(ncv)}
    for r in range(a.rounds):
        for v in range(ncv):
            _lib.check(lib.rh_commit_set_variant(v))
            for i in range(8):
                engine.commit_launch(ctx, batches[i])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(40):
                engine.commit_launch(ctx, batches[i % 8])
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 40
            cres[v].append(alg / (ms * 1e-3) / 1e9)
    _lib.check(lib.rh_commit_set_variant(14))
    for v in range(ncv):
        x = np.array(cres[v])
        print(json.dumps({"kernel": "commit", "variant": v, "median_GBps": round(float(np.median(x)), 1),
                          "min_GBps": round(float(x.min()), 1), "max_GBps": round(float(x.max()), 1),
                          "median_Gupd_s": round(float(np.median(x)) * 1e9 / alg * 1e6 / 1e9, 2)}))
    del batches
    # lease kernel variants over 8 rotating 1M-group batches (same groups and confs)
    if "lease" in only:
        now, ms, tmo = 1 << 60, 1_000_000, 100
        rng = np.random.default_rng(5)
        lb = []
        lalg = 0
        for r in range(8):
            tiers = []
            for h in host:
                ts = now - rng.integers(-ms, 3 * tmo * ms, size=h.follower.shape, dtype=np.int64)
                lin = now - rng.integers(0, 2 * tmo * ms, size=h.n, dtype=np.int64)
                if r == 0:
                    lalg += ts.size * 8 + h.n * 4 + h.n * 16 + 2 * ((h.n + 63) // 64) * 8
                t = engine.LeaseTier(follower_ts=torch.from_numpy(ts).cuda(),
                                     conf=torch.from_numpy(h.conf.view(np.int32)).cuda(),
                                     lease_in=torch.from_numpy(lin).cuda())
                tiers.append(t.alloc_outputs())
            lb.append(tiers)
        nlv = lib.rh_lease_num_variants()
        lres = {v: [] for v in range(nlv)}
        for r in range(a.rounds):
            for v in range(nlv):
                _lib.check(lib.rh_lease_set_variant(v))
                for i in range(8):
                    engine.lease_launch(ctx, lb[i], now, tmo)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(40):
                    engine.lease_launch(ctx, lb[i % 8], now, tmo)
                e1.record()
                torch.cuda.synchronize()
                lres[v].append(lalg / (e0.elapsed_time(e1) / 40 * 1e-3) / 1e9)
        _lib.check(lib.rh_lease_set_variant(2))
        for v in range(nlv):
            x = np.array(lres[v])
            print(json.dumps({"kernel": "lease", "variant": v, "median_GBps": round(float(np.median(x)), 1),
                              "min_GBps": round(float(x.min()), 1), "max_GBps": round(float(x.max()), 1)}))
    ctx.close()


if __name__ == "__main__":
    main()

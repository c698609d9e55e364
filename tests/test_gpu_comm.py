"""The multi-GPU fan-out of the C ABI (gnsship_comm_*, comm_abi.hip) and the sharded paths, on the
one-GPU box: a one-rank RCCL communicator (broadcast / all-gather / max through the real RCCL calls
on the context stream), and the sharding invariances the multi-rank runs rely on — a PRN's
acquisition result does not depend on which other PRNs share its launch, and a channel's closed
loop does not depend on which other channels share the persistent kernel (the correlating waves
follow a static schedule, so every float sum is formed in the same order): a rank's shard gives
bit-identical results to the single-GPU run, and so does a repeated run.  Multi-rank orchestration is covered with gloo on CPU
(tests/test_dist.py); RCCL refuses two ranks on one device."""
import numpy as np
import pytest

from gnss_sim_receiver_amd import abi, codes as C, engine, sharding, signals

pytestmark = pytest.mark.gpu


def test_one_rank_communicator(ctx):
    comm = engine.Comm(ctx, 1, 0, engine.comm_unique_id())
    try:
        x = (np.arange(4096, dtype=np.float32) * 0.5).view(np.uint8)
        buf = ctx.upload(x)
        comm.broadcast(buf.ptr, x.nbytes, 0)
        recv = engine.DeviceBuffer(ctx, x.nbytes)
        comm.allgather(buf.ptr, recv.ptr, x.nbytes)
        ctx.sync()
        assert np.array_equal(buf.download(np.empty_like(x)), x)
        assert np.array_equal(recv.download(np.empty_like(x)), x)
        assert comm.max_f64([1.5, -2.0]).tolist() == [1.5, -2.0]
        buf.free()
        recv.free()
    finally:
        comm.close()


def test_comm_rejects_bad_arguments(ctx):
    lib = abi.load()
    uid = engine.comm_unique_id()
    import ctypes
    h = ctypes.c_void_p()
    assert lib.gnsship_comm_create(ctx.h, 2, 2, ctypes.create_string_buffer(uid, 128), ctypes.byref(h)) == abi.E_INVAL
    assert lib.gnsship_comm_broadcast(None, None, 0, 0) == abi.E_INVAL


@pytest.mark.parametrize("world", [2, 3, 8])
def test_acquisition_prn_shards_equal_full_search(ctx, world):
    fs, n = 25000000, 25000
    sky = signals.c3_sky()
    sig = signals.generate_if(fs, n, sky, seed=0x6E550003)
    dev = ctx.upload(np.ascontiguousarray(sig))
    code = {k: C.gps_l1_ca_code_gen_complex_sampled(k + 1, fs) for k in range(32)}
    full = engine.PcpsAcquisition(ctx, fs, n, 5000, 250, 0, True, max_prns=32)
    for k in range(32):
        full.set_local_code(code[k], k)
    ref, _ = full.run(dev, n_prns=32)
    full.close()
    gathered = []
    for rank in range(world):  # each rank's launch over its PRN shard only
        mine = sharding.shard_prns(32, world, rank)
        a = engine.PcpsAcquisition(ctx, fs, n, 5000, 250, 0, True, max_prns=len(mine))
        for j, k in enumerate(mine):
            a.set_local_code(code[k], j)
        res, _ = a.run(dev, n_prns=len(mine))
        a.close()
        gathered.append(sharding.pad_rows(sharding.acq_rows(res, mine), -(-32 // world)))
    merged = sharding.merge_acq_rows(np.concatenate(gathered))
    assert sorted(merged) == list(range(32))
    for k in range(32):
        np.testing.assert_array_equal(merged[k], sharding.acq_rows([ref[k]], [k])[0])
    dev.free()


def test_closed_loop_channel_shards_equal_full_run(ctx):
    fs, vl, n_ch, n_ep = 4e6, 4000, 6, 80
    sats = signals.random_sky(n_ch, seed=51)
    x = signals.generate_if(fs, (n_ep + 3) * vl, sats, seed=52)
    dev = ctx.upload(x)
    conf = abi.TrkConf.defaults(abi.SYS_GPS_L1CA, fs, vl, rotator=abi.ROTATOR_AVX)
    for i, s in enumerate(sats):
        ctx.set_code(700 + i, s.code)

    def run(chans):
        trk = engine.DllPllVemlTracking(ctx, conf, len(chans))
        for j, c in enumerate(chans):
            s = sats[c]
            trk.start(j, 700 + c, signals.acq_delay_samples(s, fs, 0, 0), s.doppler_hz, 0, 0)
        rec, _ = trk.run(dev, 0, n_ep, n_buffer_samples=len(x))
        trk.close()
        return {c: rec[:, j] for j, c in enumerate(chans)}

    full = run(list(range(n_ch)))
    again = run(list(range(n_ch)))
    for c in range(n_ch):
        assert full[c].tobytes() == again[c].tobytes(), c  # bit-reproducible run to run
    for rank in range(2):
        part = run(sharding.shard_channels(n_ch, 2, rank))
        for c, r in part.items():
            assert r.tobytes() == full[c].tobytes(), c  # and independent of the other channels
    dev.free()

"""Multi-process channel sharding (gnss_sim_receiver_amd/sharding.py) on CPU with the gloo backend,
world_size 2: the IF block broadcast, disjoint channel shards, result gathering and max-over-ranks
timing — the same orchestration bench.py runs over RCCL.  The per-rank compute here is the CPU oracle
(test infrastructure); on the GPU box it is libgnsship.so."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gnss_sim_receiver_amd import sharding


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_channels_partition():
    for world in range(1, 9):
        for n in (0, 1, 5, 12, 64, 256):
            shards = [sharding.shard_channels(n, world, r) for r in range(world)]
            flat = sorted(c for s in shards for c in s)
            assert flat == list(range(n))
            assert max(map(len, shards)) - min(map(len, shards)) <= 1
    assert sharding.weak_channels(12, 2) == list(range(24, 36))
    with pytest.raises(ValueError):
        sharding.shard_channels(4, 2, 2)


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gnss_sim_receiver_amd import signals
    from oracle import oracle as O
    fs, vl = 4e6, 4000
    sats = signals.random_sky(6, seed=21)
    n = 5 * vl
    block = torch.zeros(n, dtype=torch.complex64)
    if rank == 0:
        block.copy_(torch.from_numpy(signals.generate_if(fs, n, sats, seed=22)))
    sharding.broadcast_block(block, src=0)
    x = block.numpy()
    mine = sharding.shard_channels(len(sats), world, rank)
    jobs = np.concatenate([signals.truth_jobs(sats[c], fs, 3, vl, [-0.25, 0, 0.25], k) for k, c in enumerate(mine)])
    res = O.corr_batch(x, jobs, [sats[c].code for c in mine])
    rows = np.concatenate([np.repeat(np.array(mine, np.float64)[:, None], 3, axis=0),
                           np.abs(res[:, :3]).astype(np.float64)], axis=1)
    gathered = sharding.gather_acq_maxima(rows)
    t = sharding.max_over_ranks(float(rank + 1))
    if rank == 0:
        np.save(os.path.join(out_dir, "gathered.npy"), gathered)
        np.save(os.path.join(out_dir, "block.npy"), x)
        np.save(os.path.join(out_dir, "tmax.npy"), np.array([t]))
    else:
        np.save(os.path.join(out_dir, "block1.npy"), x)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_broadcast_shard_gather(tmp_path, built):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    b0 = np.load(tmp_path / "block.npy")
    b1 = np.load(tmp_path / "block1.npy")
    assert np.array_equal(b0, b1)  # rank 1 received rank 0's block bit for bit
    assert float(np.load(tmp_path / "tmax.npy")[0]) == 2.0
    g = np.load(tmp_path / "gathered.npy")
    # single-process reference of the same work, channel by channel
    from gnss_sim_receiver_amd import signals
    from oracle import oracle as O
    sats = signals.random_sky(6, seed=21)
    seen = {}
    for row in g:
        seen.setdefault(int(row[0]), []).append(row[1:])
    assert sorted(seen) == list(range(6))
    for c, rows in seen.items():
        jobs = signals.truth_jobs(sats[c], 4e6, 3, 4000, [-0.25, 0, 0.25], 0)
        ref = np.abs(O.corr_batch(b0, jobs, [sats[c].code])[:, :3])
        np.testing.assert_array_equal(np.array(rows), ref.astype(np.float64))


def _acq_worker(rank, world, port, out_dir):
    """Acquisition sharded by PRN slot: the block fanned out from rank 0, every rank searches all
    bins of its PRNs (oracle compute here, libgnsship.so in bench.py), per-PRN rows all-gathered."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gnss_sim_receiver_amd import signals
    from oracle import oracle as O
    fs, n, n_slots = 4e6, 4000, 7
    block = torch.zeros(n, dtype=torch.complex64)
    if rank == 0:
        sky = signals.random_sky(3, seed=31, prns=[2, 5, 6])
        block.copy_(torch.from_numpy(signals.generate_if(fs, n, sky, seed=32)))
    sharding.broadcast_block(block, src=0)
    x = block.numpy()
    mine = sharding.shard_prns(n_slots, world, rank)
    res = [O.pcps_acquisition_core(x, O.gps_l1_ca_code_sampled(s + 1, int(fs)), int(fs), 5000, 250)[0] for s in mine]
    rows = sharding.pad_rows(sharding.acq_rows(res, mine), -(-n_slots // world))
    gathered = sharding.gather_acq_maxima(rows)
    if rank == 0:
        np.save(os.path.join(out_dir, "acq_rows.npy"), gathered)
        np.save(os.path.join(out_dir, "acq_block.npy"), x)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_acquisition_prn_shards(tmp_path, built):
    world = 2
    mp.spawn(_acq_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    g = np.load(tmp_path / "acq_rows.npy")
    x = np.load(tmp_path / "acq_block.npy")
    merged = sharding.merge_acq_rows(g)
    assert sorted(merged) == list(range(7))
    from oracle import oracle as O
    for s in range(7):  # the single-process search of every PRN, field by field
        r = O.pcps_acquisition_core(x, O.gps_l1_ca_code_sampled(s + 1, 4000000), 4000000, 5000, 250)[0]
        np.testing.assert_array_equal(merged[s], sharding.acq_rows([r], [s])[0])
    stat = {s + 1: row[6] for s, row in merged.items()}
    assert sorted(sorted(stat, key=stat.get)[-3:]) == [2, 5, 6]  # the present satellites stand out


def _trk_worker(rank, world, port, out_dir):
    """Closed-loop tracking sharded by channel: each rank runs the DLL/PLL of its channels over the
    broadcast block; epoch records gathered (oracle compute here, the persistent kernel in bench.py)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gnss_sim_receiver_amd import signals
    from oracle import trk as T
    fs, vl, n_ch, n_ep = 4e6, 4000, 4, 60
    sats = signals.random_sky(n_ch, seed=41)
    n = (n_ep + 3) * vl
    block = torch.zeros(n, dtype=torch.complex64)
    if rank == 0:
        block.copy_(torch.from_numpy(signals.generate_if(fs, n, sats, seed=42)))
    sharding.broadcast_block(block, src=0)
    x = block.numpy()
    k = T.conf("GPS", fs, vl)
    rows = []
    for c in sharding.shard_channels(n_ch, world, rank):
        s = sats[c]
        rec = T.track(k, x, s.code, signals.acq_delay_samples(s, fs, 0, 0), s.doppler_hz, 0, 0, n_ep)
        rows.append(np.stack([np.full(len(rec), c, np.float64), rec["sample_counter"].astype(np.float64), rec["carrier_doppler_hz"],
                              rec["state"].astype(np.float64)], axis=1))
    gathered = sharding.gather_acq_maxima(np.concatenate(rows))
    if rank == 0:
        np.save(os.path.join(out_dir, "trk_rows.npy"), gathered)
        np.save(os.path.join(out_dir, "trk_block.npy"), x)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_closed_loop_channel_shards(tmp_path, built):
    world = 2
    mp.spawn(_trk_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    g = np.load(tmp_path / "trk_rows.npy")
    x = np.load(tmp_path / "trk_block.npy")
    from gnss_sim_receiver_amd import signals
    from oracle import trk as T
    sats = signals.random_sky(4, seed=41)
    k = T.conf("GPS", 4e6, 4000)
    assert sorted(set(g[:, 0].astype(int))) == [0, 1, 2, 3]
    for c in range(4):
        s = sats[c]
        rec = T.track(k, x, s.code, signals.acq_delay_samples(s, 4e6, 0, 0), s.doppler_hz, 0, 0, 60)
        mine = g[g[:, 0] == c]
        np.testing.assert_array_equal(mine[:, 1], rec["sample_counter"].astype(np.float64))
        np.testing.assert_array_equal(mine[:, 2], rec["carrier_doppler_hz"])
        assert (mine[:, 3] >= 2).all()

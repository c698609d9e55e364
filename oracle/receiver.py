"""CPU restatement of the Channel role (include/gnsship_receiver.hpp) on the oracle — TEST
INFRASTRUCTURE ONLY: the checker of tools/gnsship_rx and the CPU baseline of the bench's receiver
line.  Same control logic, restated from the reference (paths relative to its root):

  ChannelFsm                channel_fsm.cc:44-220
  channel events            channel_msg_receiver_cc.cc:64-100
  set_signal / start_acq    channel.cc:215-275
  flowgraph control         gnss_flowgraph.cc: set_channels_state :2540-2564, acquisition_manager
                            :1797-1879, apply_action :1904-2009, search_next_signal :2615-2629,
                            push_back_signal :1652-1660, remove_signal :1718-1724
  acquisition block         pcps_acquisition.cc general_work :902-1031 (max_dwells 1, blocking,
                            no bit transition, no two-step grid), acquisition_core :600-871 via
                            oracle.pcps_acquisition_core, calculate_threshold :884-899
  tracking block            oracle/trk_oracle.c (dll_pll_veml_tracking.cc)

with the same deterministic schedule as the C++ core: blocks; acquisition channels in stream order
over pieces of `acq_piece` samples; then tracking over the block with a 2·vector_length tail; a loss
of lock re-acquires at the next block."""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import oracle as O
from . import trk as T


def calculate_threshold(pfa: float, fft_size: int, n_bins: int, dwells: int = 1) -> np.float32:
    """pcps_acquisition::calculate_threshold (:884-899): 2·gamma_p_inv(2·dwells, (1 − pfa)^(1/(N·nb)))."""
    from scipy.special import gammaincinv
    pfa32 = np.float32(pfa)
    p = (1.0 - float(pfa32)) ** (1.0 / float(np.float32(fft_size * n_bins)))
    return np.float32(2.0 * gammaincinv(2 * dwells, p))


@dataclass
class ReceiverConf:
    fs: int = 4000000
    channels: int = 5
    in_acquisition: int = 1
    satellite: list = field(default_factory=list)
    repeat_satellite: bool = False
    pfa: float = 0.01
    doppler_max: int = 10000
    doppler_step: int = 250
    pll_bw_hz: float = 40.0
    dll_bw_hz: float = 4.0
    order: int = 3
    pull_in_time_s: int = 10
    max_carrier_lock_fail: int = 5000
    max_code_lock_fail: int = 50
    cn0_min: int = 25
    rotator_avx: int = 1
    block_samples: int = 400000
    acq_piece: int = 8192


class _Acq:
    """One channel's pcps_acquisition block (the buffering FSM of general_work and the decision)."""

    def __init__(self, rc: ReceiverConf, threshold):
        self.rc = rc
        self.n = rc.fs // 1000  # d_consumed_samples = d_fft_size (sampled_ms = ms_per_code = 1)
        self.threshold = threshold
        self.active = False
        self.state = 0
        self.buf = np.zeros(self.n, np.complex64)
        self.count = 0
        self.sample_counter = 0
        self.code = None
        self.outcome = None

    def set_local_code(self, prn):
        self.code = O.gps_l1_ca_code_sampled(prn, self.rc.fs)

    def general_work(self, x, n):
        """Returns (consumed, event): event 1 positive, 2 negative, 0 none."""
        if not self.active:
            self.sample_counter += n
            return n, 0
        if self.state == 0:
            self.outcome = None
            self.state, self.count = 1, 0
            self.sample_counter += n
            return n, 0
        if self.state == 1:
            inc = n if n + self.count <= self.n else self.n - self.count
            self.buf[self.count:self.count + inc] = x[:inc]
            if self.count >= self.n:
                self.state = 2
            self.count += inc
            self.sample_counter += inc
            return inc, 0
        # state 2: acquisition_core + the decision (max_dwells = 1)
        r, _ = O.pcps_acquisition_core(self.buf, self.code, self.rc.fs, self.rc.doppler_max, self.rc.doppler_step)
        self.outcome = dict(delay=float(r.acq_delay_samples), doppler=float(r.doppler_hz), stamp=self.sample_counter,
                            stat=float(r.test_statistic))
        hit = np.float32(r.test_statistic) > self.threshold
        self.active = False if hit else self.active
        self.state = 0
        self.active = False
        self.count = 0
        return 0, (1 if hit else 2)


class Receiver:
    def __init__(self, rc: ReceiverConf):
        self.rc = rc
        self.n_ch = max(1, rc.channels)
        self.max_acq = min(max(0, rc.in_acquisition), self.n_ch)
        self.sat = list(rc.satellite) + [0] * (self.n_ch - len(rc.satellite))
        self.vl = rc.fs // 1000
        self.tail = 2 * self.vl
        nb = O.num_doppler_bins(rc.doppler_max, rc.doppler_step)
        thr = calculate_threshold(rc.pfa, self.vl, nb)
        self.acq = [_Acq(rc, thr) for _ in range(self.n_ch)]
        self.k = T.conf("GPS", float(rc.fs), self.vl, pll_bw_hz=rc.pll_bw_hz, dll_bw_hz=rc.dll_bw_hz, pll_filter_order=rc.order,
                        rotator_avx=rc.rotator_avx, pull_in_time_s=rc.pull_in_time_s,
                        max_carrier_lock_fail=rc.max_carrier_lock_fail, max_code_lock_fail=rc.max_code_lock_fail, cn0_min=rc.cn0_min)
        self.trk = [None] * self.n_ch
        self.fsm = [0] * self.n_ch
        self.prn = [0] * self.n_ch
        self.apos = [0] * self.n_ch
        self.available = list(range(1, 33))
        self.queue = []
        self.events = []
        self.records = [[] for _ in range(self.n_ch)]
        self.win = np.zeros(0, np.complex64)
        self.win_first = 0
        self.pos = self.now = 0
        for c in range(self.n_ch):
            self.set_signal(c, self.sat[c] if self.sat[c] else self.search_next_signal())
        self.state = [1 if c < self.max_acq else 0 for c in range(self.n_ch)]
        self.acq_count = self.max_acq
        for c in range(self.n_ch):
            if self.state[c] == 1:
                self.ev_start_acquisition(c)
        self.drain()

    # ---- ChannelFsm events and actions ----
    def ev_start_acquisition(self, c):
        if self.fsm[c] in (1, 2):
            return False
        self.fsm[c] = 1
        self.act_start_acquisition(c)
        return True

    def ev_valid_acquisition(self, c):
        if self.fsm[c] != 1:
            return False
        self.fsm[c] = 2
        o = self.acq[c].outcome
        self.trk[c] = T.Channel(self.k, O.gps_l1_ca_code(self.prn[c]), o["delay"], o["doppler"], o["stamp"], self.now, prn=self.prn[c])
        self.queue.append((c, 1))
        return True

    def ev_failed_acquisition(self, c):
        if self.fsm[c] != 1:
            return False
        if self.rc.repeat_satellite:
            self.act_start_acquisition(c)
        else:
            self.fsm[c] = 3
            self.queue.append((c, 0))
        return True

    def ev_failed_tracking_standby(self, c):
        if self.fsm[c] != 2:
            return False
        self.fsm[c] = 0
        self.queue.append((c, 2))
        return True

    def act_start_acquisition(self, c):
        a = self.acq[c]
        a.active = False
        if a.sample_counter < self.now:
            a.sample_counter = self.now
        a.active = True
        self.apos[c] = self.now
        self.events.append((self.now, c, 3, self.prn[c], 0.0, 0.0, 0.0))

    # ---- Channel / flowgraph ----
    def set_signal(self, c, prn):
        self.prn[c] = prn
        self.acq[c].set_local_code(prn)

    def search_next_signal(self):
        p = self.available.pop(0)
        self.available.append(p)
        return p

    def push_back_signal(self, p):
        if p in self.available:
            self.available.remove(p)
        self.available.append(p)

    def acquisition_manager(self, who):
        for i in range(self.n_ch):
            cc = (i + who + 1) % self.n_ch
            if self.acq_count < self.max_acq and self.state[cc] == 0:
                self.set_signal(cc, self.prn[cc] if self.sat[cc] else self.search_next_signal())
                self.state[cc] = 1
                self.acq_count += 1
                self.ev_start_acquisition(cc)

    def apply_action(self, who, what):
        gs = self.prn[who]
        if what == 0:
            self.state[who] = 0
            self.acq_count = max(0, self.acq_count - 1)
            self.acquisition_manager(who)
            if self.sat[who] == 0:
                self.push_back_signal(gs)
        elif what == 1:
            if gs in self.available:
                self.available.remove(gs)
            self.state[who] = 2
            self.acq_count = max(0, self.acq_count - 1)
            self.acquisition_manager(who)
        elif what == 2:
            if self.acq_count < self.max_acq:
                self.state[who] = 1
                self.acq_count += 1
                self.set_signal(who, gs)
                self.ev_start_acquisition(who)
            else:
                self.state[who] = 0
                if self.sat[who] == 0:
                    self.push_back_signal(gs)

    def drain(self):
        while self.queue:
            self.apply_action(*self.queue.pop(0))

    # ---- the stream ----
    def work(self, x: np.ndarray):
        x = np.ascontiguousarray(x, np.complex64)
        i = 0
        while i < len(x):
            m = min(len(x) - i, self.rc.block_samples)
            self._block(x[i:i + m])
            i += m

    def _block(self, x):
        b0, b1 = self.pos, self.pos + len(x)
        while True:
            cands = [c for c in range(self.n_ch) if self.fsm[c] == 1 and self.apos[c] < b1]
            if not cands:
                break
            c = min(cands, key=lambda i: (self.apos[i], i))
            p = self.apos[c]
            m = int(min(self.rc.acq_piece, b1 - p))
            used, ev = self.acq[c].general_work(x[p - b0:p - b0 + m], m)
            if used == 0 and ev == 0:
                used, ev = self.acq[c].general_work(x[p - b0:p - b0 + m], m)
                if used == 0 and ev == 0:
                    self.apos[c] = b1
                    continue
            self.apos[c] = p + used
            self.now = self.apos[c]
            if ev:
                o = self.acq[c].outcome
                self.events.append((self.now, c, 1 if ev == 1 else 0, self.prn[c], o["doppler"], o["delay"], o["stat"]))
                if ev == 1:
                    self.ev_valid_acquisition(c)
                else:
                    self.ev_failed_acquisition(c)
                self.drain()
        keep = min(self.tail, b0 - self.win_first)
        self.win = np.concatenate([self.win[len(self.win) - keep:] if keep else self.win[:0], x])
        self.win_first = b0 - keep
        for c in range(self.n_ch):
            if self.fsm[c] != 2 or self.trk[c] is None:
                continue
            rec = self.trk[c].run(self.win, self.win_first, len(self.win) // (self.vl - 1) + 2)
            self.records[c].extend(rec.tolist())
            if len(rec) and (rec["flags"] & 2).any():
                self.now = b1
                self.events.append((b1, c, 2, self.prn[c], 0.0, 0.0, 0.0))
                self.trk[c] = None
                self.ev_failed_tracking_standby(c)
                self.drain()
        self.pos = self.now = b1

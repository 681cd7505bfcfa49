"""The packet-buffer lifecycle of the Go batch managers, replayed on a model (CPU, no device).

go/internal/fec/batch_manager_hip.go hands registered packet buffers (packet_pool_hip.go) to the
device by reference and must give every one back to the process-wide pool: a payload a block keeps
after its block's data (or frames) are polled, one no block keeps at the next PollRecovered, and
everything still held at connection close. There is no Go toolchain here, so this test restates
that bookkeeping statement for statement (line numbers below) over the reference's block rules
(block.go:56-95: a duplicate SSID / ParityID is ignored; complete = all k sources; recoverable =
sources + repairs >= k) and replays connections against it: lossless streams, losses, duplicates,
blocks completed by sources after repairs, unrecoverable blocks, an exhausted pool (heap payloads),
and close mid-stream. It checks that the pool ends full, that no buffer goes back twice, and that
no buffer goes back while the device or the connection may still read it. It also replays the
destination connection ID each staged block carries to the frames recovered from it
(fec_poll.go RecoveredBlock, connection.go.diff handleRecoveredFEC) against the reference's
RETIRE_CONNECTION_ID check (conn_id_generator.go:70-89, connection.go:1443-1444,1605-1606)."""
import random

import pytest


class Buf:
    """One packet buffer; pool is None for a heap buffer (Put ignores those)."""

    def __init__(self, pool=None):
        self.pool = pool


class Pool:
    """packet_pool_hip.go: Get (None when exhausted), Put (heap buffers ignored)."""

    def __init__(self, n):
        self.free = [Buf(self) for _ in range(n)]
        self.out = set()
        self.n = n

    def get(self):
        if not self.free:
            return None
        b = self.free.pop()
        self.out.add(b)
        return b

    def put(self, b):
        if b.pool is not self:
            return
        assert b in self.out, "buffer returned twice"
        self.out.remove(b)
        self.free.append(b)

    def must_be_out(self, bufs, who):
        for b in bufs:
            assert b.pool is not self or b in self.out, "%s reads a buffer already back in the pool" % who


class Block:
    def __init__(self, bid, k):
        self.id, self.k = bid, k
        self.src, self.rep = {}, {}

    def add_source(self, ssid, buf):          # block.go:56-70 (duplicates ignored)
        self.src.setdefault(ssid, buf)

    def add_repair(self, pid, buf):           # block.go:73-85
        self.rep.setdefault(pid, buf)

    def complete(self):                       # block.go:93-95
        return len(self.src) == self.k

    def recoverable(self):                    # block.go:88-90
        return len(self.src) + len(self.rep) >= self.k

    def payloads(self):                       # batch_manager_hip.go:259-268 blockPayloads
        return list(self.src.values()) + list(self.rep.values())


class Device:
    """The library side of BatchReceiver / BatchSender by reference: a submitted block's buffers are
    read when its batch is coded, i.e. at some poll after the submit."""

    def __init__(self, pool, rng):
        self.pool, self.rng, self.inflight = pool, rng, []

    def submit(self, bid, bufs):
        self.inflight.append((bid, list(bufs)))

    def poll(self, wait, max_blocks=None):
        n = len(self.inflight) if wait else self.rng.randint(0, len(self.inflight))
        if max_blocks is not None:
            n = min(n, max_blocks)
        done, self.inflight = self.inflight[:n], self.inflight[n:]
        for _, bufs in done:
            self.pool.must_be_out(bufs, "the device")
        return [bid for bid, _ in done]

    def close(self):   # fec_go_*_free waits for a batch in flight: the device reads it
        for _, bufs in self.inflight:
            self.pool.must_be_out(bufs, "the device (close)")
        self.inflight = []


class Receiver:
    """batchManager, receive side with the pool (rxHeld != nil)."""

    def __init__(self, k, pool, dev):
        self.k, self.pool, self.rx = k, pool, dev
        self.status = {}          # bid -> [block or None, processed]
        self.pending = 0
        self.rx_held = {}
        self.release = []
        self.repair_dest = None   # :115-116 repairDest, dest
        self.dest = {}

    def _status(self, bid):
        return self.status.setdefault(bid, [Block(bid, self.k), False])

    def set_repair_dest(self, cid):   # SetRepairDestConnID
        self.repair_dest = cid

    def handle_source(self, ssid, buf):   # :272-292 over manager.go:200-227
        bid = ssid // self.k
        prev = self.status[bid][0] if bid in self.status else None
        st = self._status(bid)
        ret = None
        if not st[1]:
            st[0].add_source(ssid, buf)
            if st[0].complete():
                st[0], st[1] = None, True
            ret = buf
        cur = st[0]
        if cur is not None:
            if cur.src.get(ssid) is not buf:
                self.release.append(buf)
        elif prev is not None:   # completed by this symbol: the block is dropped
            if prev.src.get(ssid) is not buf:
                self.release.append(buf)
            self.release.extend(prev.payloads())
        else:
            self.release.append(buf)
        return ret

    def handle_repair(self, bid, pid, buf):   # :298-347
        st = self._status(bid)
        if st[1]:
            self.release.append(buf)
            return
        st[0].add_repair(pid, buf)
        if st[0].rep.get(pid) is not buf:
            self.release.append(buf)
        if st[0].recoverable():
            staged = not st[0].complete()   # fec_go_decoder_submit_ref stages only what has a loss
            if staged:
                self.rx.submit(bid, st[0].payloads())
                self.pending += 1
                self.dest[bid] = self.repair_dest
                self.rx_held[bid] = st[0].payloads()
            else:
                self.release.extend(st[0].payloads())
            st[0], st[1] = None, True

    def poll_recovered(self, wait):   # :356-386: [(block, destConnID)] in staging order
        out = []
        for b in self.release:
            self.pool.put(b)
        self.release = []
        while self.pending > 0:
            rec = self.rx.poll(wait)
            for bid in rec:
                out.append((bid, self.dest.pop(bid)))
                for b in self.rx_held.pop(bid):
                    self.pool.put(b)
            self.pending -= len(rec)
            if not wait or not rec:
                break
        return out

    def recovery_pending(self):   # :391
        return self.pending > 0 or len(self.release) > 0

    def close(self):   # :402-438
        self.rx.close()
        self.dest = {}
        for bufs in self.rx_held.values():
            for b in bufs:
                self.pool.put(b)
        self.rx_held = {}
        for b in self.release:
            self.pool.put(b)
        self.release = []
        for st in self.status.values():
            if st[0] is not None:
                for b in st[0].payloads():
                    self.pool.put(b)


class Sender:
    """batchManager, send side with the pool (held != nil)."""

    def __init__(self, k, m, pool, dev):
        self.k, self.m, self.pool, self.tx = k, m, pool, dev
        self.status = {}
        self.held = {}

    def add_source(self, ssid, buf):   # :155-192
        bid = ssid // self.k
        st = self.status.setdefault(bid, [Block(bid, self.k), False])
        if st[1]:
            return
        st[0].add_source(ssid, buf)
        if st[0].complete():
            self.tx.submit(bid, st[0].src.values())
            self.held[bid] = list(st[0].src.values())
            st[0], st[1] = None, True

    def poll_repair_frames(self, max_frames):   # :197-218
        for bid in self.tx.poll(False, max_frames // self.m if max_frames > 0 else 0):
            for b in self.held.pop(bid):
                self.pool.put(b)

    def close(self):   # :402-438
        self.tx.close()
        for bufs in self.held.values():
            for b in bufs:
                self.pool.put(b)
        self.held = {}
        for st in self.status.values():
            if st[0] is not None:
                for b in st[0].payloads():
                    self.pool.put(b)


def _payload(pool):
    """wire.FECPayloadBuffer (batch_manager_hip.go:235-250): a pool buffer, or the heap when the
    pool is exhausted."""
    return pool.get() or Buf(None)


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("k,m,pool_size", [(8, 4, 4096), (20, 10, 4096), (8, 4, 37)])
def test_receiver_returns_every_buffer(seed, k, m, pool_size):
    rng = random.Random(seed * 1000 + k + pool_size)
    pool = Pool(pool_size)
    rcv = Receiver(k, pool, Device(pool, rng))
    loss = [0.0, 0.1, 0.3][seed % 3]
    nblocks = 60
    stop = nblocks if seed % 4 else rng.randint(5, nblocks)   # some connections close mid-stream
    events = []
    for bid in range(stop):
        for j in range(k):
            if rng.random() >= loss:
                events.append(("s", bid * k + j))
                if rng.random() < 0.05:
                    events.append(("s", bid * k + j))          # a duplicate source
        for p in range(m):
            if rng.random() >= loss:
                events.append(("r", bid, p))
                if rng.random() < 0.05:
                    events.append(("r", bid, p))               # a duplicate repair
    # light reordering: a source may arrive after its block's repairs
    for i in range(len(events) - 1):
        if rng.random() < 0.1:
            events[i], events[i + 1] = events[i + 1], events[i]
    i = 0
    while i < len(events):
        burst = events[i:i + rng.randint(1, 8)]
        i += len(burst)
        for ev in burst:
            buf = _payload(pool)
            if ev[0] == "s":
                got = rcv.handle_source(ev[1], buf)
                if got is not None:   # the connection parses the payload after the call
                    pool.must_be_out([got], "the frame parser")
            else:
                rcv.handle_repair(ev[1], ev[2], buf)
        if rcv.recovery_pending():   # connection.go.diff handleRecoveredFEC(false)
            rcv.poll_recovered(False)
    if seed % 2 == 0 and rcv.recovery_pending():   # a final drain before close, or none
        rcv.poll_recovered(True)
    rcv.close()
    assert not pool.out and len(pool.free) == pool.n


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("k,m,pool_size", [(8, 4, 4096), (20, 10, 4096), (8, 4, 29)])
def test_sender_returns_every_buffer(seed, k, m, pool_size):
    rng = random.Random(seed * 77 + k + pool_size)
    pool = Pool(pool_size)
    snd = Sender(k, m, pool, Device(pool, rng))
    n = k * rng.randint(3, 40) + rng.randint(0, k - 1)   # the last block may stay incomplete
    for ssid in range(n):
        snd.add_source(ssid, _payload(pool))   # the packer builds the payload in the pool buffer
        if rng.random() < 0.3:
            snd.poll_repair_frames(rng.choice([0, m, 3 * m, 64]))
    snd.close()
    assert not pool.out and len(pool.free) == pool.n


class ProtocolViolation(Exception):
    pass


class ConnIDGenerator:
    """conn_id_generator.go:70-89 Retire: retiring the connection ID the packet carrying the
    frame was sent to is a PROTOCOL_VIOLATION; a sequence number no longer active is ignored."""

    def __init__(self, active):
        self.active = dict(active)   # seq -> connection ID
        self.highest = max(active)

    def retire(self, seq, sent_with):
        if seq > self.highest:
            raise ProtocolViolation("retired connection ID %d (highest issued: %d)" % (seq, self.highest))
        cid = self.active.get(seq)
        if cid is None:
            return
        if cid == sent_with:
            raise ProtocolViolation("retired connection ID %d (%s), which was used as the Destination "
                                    "Connection ID on this packet" % (seq, cid))
        del self.active[seq]


def _replay_retires(packets, per_block):
    """Packets [(destConnID, block, retire_seq)], each carrying the REPAIR frame that makes its block
    recoverable; the block's recovered frames hold RETIRE_CONNECTION_ID(retire_seq). The blocks
    decode on the device and are handed over after every packet has been handled (one receive
    burst, connection.go.diff run loop). per_block: each block's frames with the ID its block carries
    (RecoveredBlock.DestConnID); else with one per-connection ID that every REPAIR frame overwrites
    (the round-4 fecDestConnID)."""
    k = 4
    pool = Pool(256)
    rcv = Receiver(k, pool, Device(pool, random.Random(1)))
    gen = ConnIDGenerator({0: "A", 1: "B", 2: "C"})
    last_dest = None
    retire_of = {}
    for dest, bid, seq in packets:
        for j in range(1, k):                  # sources 1..k-1 arrive, source 0 is lost
            rcv.handle_source(bid * k + j, _payload(pool))
        rcv.set_repair_dest(dest)              # connection.go.diff, case *wire.RepairFrame
        last_dest = dest
        rcv.handle_repair(bid, 0, _payload(pool))
        retire_of[bid] = seq
    got = rcv.poll_recovered(True)
    assert [b for b, _ in got] == [b for _, b, _ in packets]   # staging order
    for bid, dest in got:
        gen.retire(retire_of[bid], dest if per_block else last_dest)
    rcv.close()
    assert not pool.out
    return gen


def test_recovered_frames_carry_their_packets_dest_conn_id():
    # block 0 staged by a packet sent to A retires B; block 1 staged by a packet sent to B retires C:
    # both are legal in the reference, which handles each block's frames inside its own packet
    gen = _replay_retires([("A", 0, 1), ("B", 1, 2)], per_block=True)
    assert gen.active == {0: "A"}
    # one per-connection ID overwritten by the last REPAIR frame (B) makes block 0's retire of B look
    # like retiring the packet's own destination: a spurious PROTOCOL_VIOLATION
    with pytest.raises(ProtocolViolation):
        _replay_retires([("A", 0, 1), ("B", 1, 2)], per_block=False)


def test_recovered_retire_of_own_dest_is_still_a_violation():
    # the reference's check is kept: a block staged by a packet sent to B that retires B
    with pytest.raises(ProtocolViolation):
        _replay_retires([("A", 0, 2), ("B", 1, 1)], per_block=True)

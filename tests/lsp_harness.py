"""Fake LSP server for tests -- TEST INFRASTRUCTURE ONLY.

A small restatement of the server side of the reference's LSP transport
(cmu440/ = p1/src/github.com/cmu440/), enough to drive native clients the way
the staff `mtest` binary drives a miner (p1/README.md:139-141):

* lsp.Message JSON (lsp/message.go:20-27; Payload base64, nil -> null)
* checksum: 16-bit end-around-carry sum, not complemented
  (lsp/client_impl.go:183-198, lsp/checksum.go:10-47)
* Connect -> Ack(connID, 0), repeated for a duplicate Connect
  (server_impl.go:292-335)
* Data acked on receipt and delivered in SeqNum order; own Data resent every
  epoch until acked, WindowSize in flight (server_impl.go:365-392)
* liveness timers as the reference server keeps them per client
  (server_impl.go:397-420): any intact message resets them; a reminder
  Ack(connID, 0) goes out after one epoch with nothing received (and every
  epoch after that); nothing received for EpochLimit epochs drops the client.
  heartbeat="spec" instead sends the reminder in every epoch in which the
  server sent nothing, as the LSP handout words it.

Optional random datagram loss in either direction, like lspnet's
SetWriteDropPercent/SetReadDropPercent (lspnet/staff.go).
"""
from __future__ import annotations

import base64
import json
import queue
import random
import socket
import threading
import time


def int_sum(v: int) -> int:
    u = v & 0xFFFFFFFF
    return (u & 0xFFFF) + (u >> 16)


def checksum(conn_id: int, seq: int, size: int, payload: bytes) -> int:
    s = int_sum(conn_id) + int_sum(seq) + int_sum(size)
    for i in range(0, len(payload), 2):
        lo = payload[i]
        hi = payload[i + 1] if i + 1 < len(payload) else 0
        s += lo | (hi << 8)
    while s > 0xFFFF:
        s = (s >> 16) + (s & 0xFFFF)
    return s


CONNECT, DATA, ACK = 0, 1, 2


def encode(typ: int, conn_id: int, seq: int, payload: bytes | None) -> bytes:
    size = len(payload) if payload is not None else 0
    cs = checksum(conn_id, seq, size, payload) if payload is not None else 0
    p = "null" if payload is None else '"' + base64.b64encode(payload).decode() + '"'
    return ('{"Type":%d,"ConnID":%d,"SeqNum":%d,"Size":%d,"Checksum":%d,"Payload":%s}'
            % (typ, conn_id, seq, size, cs, p)).encode()


def decode(data: bytes):
    try:
        o = {k.lower(): v for k, v in json.loads(data).items()}
        payload = o.get("payload")
        payload = base64.b64decode(payload, validate=True) if payload is not None else None
        return (int(o.get("type", 0)), int(o.get("connid", 0)), int(o.get("seqnum", 0)),
                int(o.get("size", 0)), int(o.get("checksum", 0)), payload)
    except Exception:
        return None


class _Client:
    def __init__(self, conn_id, addr):
        self.conn_id, self.addr = conn_id, addr
        self.expected, self.next_seq = 1, 1
        self.inflight = {}        # seq -> bytes
        self.backlog = []         # (seq, bytes)
        self.pending = {}
        self.ready = queue.Queue()
        self.last_rx = time.monotonic()
        self.remind_at = self.last_rx
        self.sent = False          # anything sent this epoch (heartbeat="spec")
        self.lost = False


class FakeLspServer:
    def __init__(self, epoch_ms=100, epoch_limit=5, window=1, drop_send=0.0, drop_recv=0.0, seed=0,
                 heartbeat="reference"):
        assert heartbeat in ("reference", "spec")
        self.heartbeat = heartbeat
        self.epoch, self.limit, self.window = epoch_ms / 1000.0, epoch_limit, window
        self.drop_send, self.drop_recv = drop_send, drop_recv
        self.rng = random.Random(seed)
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.sock.bind(("127.0.0.1", 0))
        self.sock.settimeout(0.01)
        self.port = self.sock.getsockname()[1]
        self.hostport = f"127.0.0.1:{self.port}"
        self.lock = threading.Lock()
        self.by_addr, self.by_id = {}, {}
        self.new_conns = queue.Queue()
        self.next_id = 1
        self.stopping = False
        self.th = threading.Thread(target=self._loop, daemon=True)
        self.th.start()

    # -- public API -----------------------------------------------------------
    def accept(self, timeout=30.0) -> int:
        return self.new_conns.get(timeout=timeout)

    def read(self, conn_id: int, timeout=60.0) -> bytes:
        return self.by_id[conn_id].ready.get(timeout=timeout)

    def write(self, conn_id: int, payload: bytes):
        with self.lock:
            c = self.by_id[conn_id]
            seq = c.next_seq
            c.next_seq += 1
            c.backlog.append((seq, encode(DATA, conn_id, seq, payload)))
            self._pump(c)

    def is_lost(self, conn_id: int) -> bool:
        return self.by_id[conn_id].lost

    def close(self):
        self.stopping = True
        self.th.join(timeout=5)
        self.sock.close()

    # -- internals -------------------------------------------------------------
    def _send(self, data: bytes, addr):
        c = self.by_addr.get(addr)
        if c is not None:
            c.sent = True
        if self.drop_send and self.rng.random() < self.drop_send:
            return
        try:
            self.sock.sendto(data, addr)
        except OSError:
            pass

    def _pump(self, c: _Client):
        while c.backlog:
            lowest = min(c.inflight) if c.inflight else c.backlog[0][0]
            seq, data = c.backlog[0]
            if seq >= lowest + self.window:
                break
            c.backlog.pop(0)
            c.inflight[seq] = data
            self._send(data, c.addr)

    def _loop(self):
        next_epoch = time.monotonic() + self.epoch
        while not self.stopping:
            try:
                data, addr = self.sock.recvfrom(65536)
            except socket.timeout:
                data = None
            except OSError:
                return
            if data is not None and not (self.drop_recv and self.rng.random() < self.drop_recv):
                self._handle(data, addr)
            self._timers()
            if time.monotonic() >= next_epoch:
                next_epoch += self.epoch
                self._tick()

    def _handle(self, data, addr):
        m = decode(data)
        if m is None:
            return
        typ, conn_id, seq, size, cs, payload = m
        with self.lock:
            c = self.by_addr.get(addr)
            if typ == DATA:
                if payload is None or len(payload) < size:
                    return
                payload = payload[:size]
                if checksum(conn_id, seq, size, payload) != cs:
                    return
            if typ == CONNECT and c is None:
                c = _Client(self.next_id, addr)
                self.next_id += 1
                self.by_addr[addr] = c
                self.by_id[c.conn_id] = c
                self.new_conns.put(c.conn_id)
            if c is not None and not c.lost:             # gotMessageChan: reset both timers
                c.last_rx = time.monotonic()
                c.remind_at = c.last_rx + self.epoch
            if typ == CONNECT:
                self._send(encode(ACK, c.conn_id, 0, None), addr)
            elif c is None:
                return
            elif typ == DATA:
                self._send(encode(ACK, c.conn_id, seq, None), addr)
                if seq == c.expected:
                    c.ready.put(payload)
                    c.expected += 1
                    while c.expected in c.pending:
                        c.ready.put(c.pending.pop(c.expected))
                        c.expected += 1
                elif seq > c.expected:
                    c.pending.setdefault(seq, payload)
            elif typ == ACK and seq > 0:
                if c.inflight.pop(seq, None) is not None:
                    self._pump(c)

    def _timers(self):
        """connDropTimer and (reference mode) reminderTimer, server_impl.go:397-420."""
        now = time.monotonic()
        with self.lock:
            for c in self.by_id.values():
                if c.lost:
                    continue
                if now - c.last_rx >= self.epoch * self.limit:
                    c.lost = True
                elif self.heartbeat == "reference" and now >= c.remind_at:
                    self._send(encode(ACK, c.conn_id, 0, None), c.addr)
                    c.remind_at = now + self.epoch

    def _tick(self):
        with self.lock:
            for c in self.by_id.values():
                if c.lost:
                    continue
                for data in c.inflight.values():
                    self._send(data, c.addr)
                if self.heartbeat == "spec" and not c.sent:
                    self._send(encode(ACK, c.conn_id, 0, None), c.addr)
                c.sent = False

"""Mirror of the reference's ``bitcoin`` package (the miner's app contract).

Reference (cmu440/ = p1/src/github.com/cmu440/):
  * ``Message``, ``MsgType``, ``NewRequest``/``NewResult``/``NewJoin``,
    ``String`` -- cmu440/bitcoin/message.go:7-62
  * ``Hash`` -- cmu440/bitcoin/hash.go:13-17 (here: ``hm_hash`` of
    libhipminer.so, host SHA-256; the GPU path is the scan, not single hashes)
  * ``marshal``/``unmarshal`` -- the apps' json.Marshal/json.Unmarshal of a
    Message (miner/miner.go:11-19): field order Type, Data, Lower, Upper,
    Hash, Nonce; Go's encoding/json string escaping (HTML-safe: <, >, & as
    \\u003c/\\u003e/\\u0026; U+2028/U+2029 escaped; invalid UTF-8 -> U+FFFD;
    control characters as \\u00XX except \\n \\r \\t, the go1.10 form).
"""
from __future__ import annotations

import json
from dataclasses import dataclass

from . import _lib

MAXU64 = (1 << 64) - 1

# MsgType (message.go:9-13)
Join, Request, Result = 0, 1, 2
_TYPE_NAMES = {Join: "Join", Request: "Request", Result: "Result"}


@dataclass
class Message:
    """bitcoin.Message (message.go:18-23).  Data is kept as Go string bytes."""
    Type: int = Join
    Data: bytes = b""
    Lower: int = 0
    Upper: int = 0
    Hash: int = 0
    Nonce: int = 0

    def String(self) -> str:  # message.go:47-62
        d = self.Data.decode("utf-8", "replace")
        if self.Type == Request:
            return f"[Request {d} {self.Lower} {self.Upper}]"
        if self.Type == Result:
            return f"[Result {self.Hash} {self.Nonce}]"
        if self.Type == Join:
            return "[Join]"
        return ""

    __str__ = String


def NewRequest(data, lower: int, upper: int) -> Message:  # message.go:27-34
    return Message(Type=Request, Data=_lib.as_bytes(data), Lower=lower, Upper=upper)


def NewResult(hash_: int, nonce: int) -> Message:  # message.go:38-44
    return Message(Type=Result, Hash=hash_, Nonce=nonce)


def NewJoin() -> Message:  # message.go:47-49
    return Message(Type=Join)


def Hash(msg, nonce: int) -> int:
    """bitcoin.Hash(msg, nonce) (hash.go:13-17) via hm_hash."""
    return _lib.host_hash(msg, nonce)


# ---- JSON wire form (encoding/json) ------------------------------------------

def _decode_rune(b: bytes, i: int):
    """utf8.DecodeRune: (rune, size), or (None, 1) for an invalid byte."""
    c = b[i]
    size = 2 if 0xC2 <= c <= 0xDF else 3 if 0xE0 <= c <= 0xEF else 4 if 0xF0 <= c <= 0xF4 else 0
    if size == 0 or i + size > len(b):
        return None, 1
    try:
        ch = b[i:i + size].decode("utf-8")  # strict: rejects overlongs and surrogates
    except UnicodeDecodeError:
        return None, 1
    return ord(ch), size


def _go_json_string(b: bytes) -> str:
    """encoding/json string encoding (escapeHTML on) of Go string bytes."""
    out = ['"']
    i, n = 0, len(b)
    while i < n:
        c = b[i]
        if c < 0x80:
            ch = chr(c)
            if ch == '"':
                out.append('\\"')
            elif ch == "\\":
                out.append("\\\\")
            elif ch == "\n":
                out.append("\\n")
            elif ch == "\r":
                out.append("\\r")
            elif ch == "\t":
                out.append("\\t")
            elif c < 0x20 or ch in "<>&":
                out.append("\\u%04x" % c)
            else:
                out.append(ch)
            i += 1
            continue
        r, size = _decode_rune(b, i)
        if r is None:
            out.append("\\ufffd")  # invalid UTF-8 byte
        elif r in (0x2028, 0x2029):
            out.append("\\u%04x" % r)
        else:
            out.append(chr(r))
        i += size
    out.append('"')
    return "".join(out)


def marshal(m: Message) -> bytes:
    """json.Marshal(*bitcoin.Message)."""
    body = ('{"Type":%d,"Data":%s,"Lower":%d,"Upper":%d,"Hash":%d,"Nonce":%d}'
            % (m.Type, _go_json_string(m.Data), m.Lower, m.Upper, m.Hash, m.Nonce))
    return body.encode("utf-8")


def _fix_surrogates(s: str) -> str:
    # Go's decoder maps unpaired UTF-16 surrogate escapes to U+FFFD
    return "".join("�" if 0xD800 <= ord(c) <= 0xDFFF else c for c in s)


def unmarshal(data: bytes) -> tuple[Message, Exception | None]:
    """json.Unmarshal into a zero Message: case-insensitive keys, unknown keys
    ignored, the error returned (the miner ignores it, miner.go:45)."""
    m = Message()
    try:
        # Go replaces invalid UTF-8 in JSON strings with U+FFFD
        text = data.decode("utf-8", "replace") if isinstance(data, (bytes, bytearray)) else data
        obj = json.loads(text)
    except (ValueError, UnicodeDecodeError) as e:
        return m, e
    if not isinstance(obj, dict):
        return m, ValueError("json: cannot unmarshal non-object into Message")
    err = None
    fields = {f.lower(): f for f in ("Type", "Data", "Lower", "Upper", "Hash", "Nonce")}
    for k, v in obj.items():
        f = fields.get(k.lower())
        if f is None:
            continue
        if f == "Data":
            if isinstance(v, str):
                m.Data = _fix_surrogates(v).encode("utf-8")
            elif v is not None:
                err = err or ValueError("json: cannot unmarshal into Message.Data")
        else:
            if isinstance(v, bool) or not isinstance(v, int):
                if v is not None:
                    err = err or ValueError(f"json: cannot unmarshal into Message.{f}")
                continue
            lim = (1 << 63) - 1 if f == "Type" else MAXU64
            low = -(1 << 63) if f == "Type" else 0
            if not low <= v <= lim:
                err = err or ValueError(f"json: value out of range for Message.{f}")
                continue
            setattr(m, f, v)
    return m, err

"""Host mirror of the reference interface: Message JSON wire form (message.go +
encoding/json), the miner's Request -> Result step (miner.go:44-62) with its
Upper+1 wrap, and the planner's segment layouts."""
import pytest

from distributed_bitcoinminer_amd import _lib, bitcoin, miner

MAX = (1 << 64) - 1


def test_marshal_field_order_and_values():
    req = bitcoin.NewRequest("bradfitz", 0, 9999)
    assert bitcoin.marshal(req) == (b'{"Type":1,"Data":"bradfitz","Lower":0,"Upper":9999,'
                                    b'"Hash":0,"Nonce":0}')
    res = bitcoin.NewResult(356393768206, 7645578)
    assert bitcoin.marshal(res) == (b'{"Type":2,"Data":"","Lower":0,"Upper":0,'
                                    b'"Hash":356393768206,"Nonce":7645578}')
    assert bitcoin.marshal(bitcoin.NewJoin()) == (b'{"Type":0,"Data":"","Lower":0,"Upper":0,'
                                                  b'"Hash":0,"Nonce":0}')
    big = bitcoin.NewRequest("x", MAX - 1, MAX)
    assert b'"Lower":18446744073709551614,"Upper":18446744073709551615' in bitcoin.marshal(big)


def test_marshal_go_string_escaping():
    m = bitcoin.NewRequest(b'a<b>&"\\\n\r\t\x01\x7f\xe2\x80\xa8\xff\xc3\xa9', 0, 0)
    data = bitcoin.marshal(m)
    expect = ('"a\\u003cb\\u003e\\u0026\\"\\\\\\n\\r\\t\\u0001\x7f\\u2028\\ufffdé"')
    assert expect.encode("utf-8") in data


def test_unmarshal_roundtrip_and_go_rules():
    for d in [b"bradfitz", b"", "thom yorke".encode(), "é中".encode(), b"<&>"]:
        m = bitcoin.NewRequest(d, 5, 10**19)
        back, err = bitcoin.unmarshal(bitcoin.marshal(m))
        assert err is None and back == m
    m, err = bitcoin.unmarshal(b'{"type":1,"DATA":"x","lower":3,"Upper":4,"extra":7}')
    assert err is None and (m.Type, m.Data, m.Lower, m.Upper) == (1, b"x", 3, 4)
    m, err = bitcoin.unmarshal(b'{"Data":"\\ud800"}')
    assert m.Data == "�".encode()
    m, err = bitcoin.unmarshal(b"not json")
    assert err is not None and m == bitcoin.Message()


def test_string_form():
    assert bitcoin.NewRequest("a", 1, 2).String() == "[Request a 1 2]"
    assert bitcoin.NewResult(3, 4).String() == "[Result 3 4]"
    assert bitcoin.NewJoin().String() == "[Join]"


def test_hash_matches_reference_examples():
    assert bitcoin.Hash("thom yorke", 19970521) == 1397265185016851828  # p1/README.md:105 call
    assert bitcoin.Hash("bradfitz", 0) == 12865759911151091764


def test_eval_range_wrap_quirk():
    assert miner.eval_range(0, 9999) == (0, 9999)
    assert miner.eval_range(5, 4) is None
    assert miner.eval_range(MAX - 5, MAX) is None   # upper := Upper+1 wraps to 0
    assert miner.eval_range(MAX, MAX) is None
    assert miner.eval_range(MAX - 5, MAX - 1) == (MAX - 5, MAX - 1)


class _OracleCtx:
    """Test double for the GPU context: the CPU oracle (tests only)."""

    def __init__(self, oracle_mod):
        self.o = oracle_mod

    def scan(self, data, lo, hi):
        return self.o.c_scan(data, lo, hi, threads=2)


def test_eval_request_logic(oracle_mod, golden):
    mnr = miner.Miner(ctx=_OracleCtx(oracle_mod))
    for k in golden["miner_eval_kats"]:
        req = bitcoin.NewRequest(bytes.fromhex(k["msg_hex"]), int(k["lower"]), int(k["upper"]))
        out, err = bitcoin.unmarshal(mnr.eval_request(bitcoin.marshal(req)))
        assert err is None and out.Type == bitcoin.Result
        assert (out.Hash, out.Nonce) == (int(k["hash"]), int(k["nonce"]))


# ---- planner -------------------------------------------------------------------

def _digits(n):
    return len(str(n))


@pytest.mark.parametrize("L", list(range(0, 140)) + [200, 1000])
def test_planner_layouts(L):
    msg = bytes((i * 7 + 1) % 256 for i in range(L))
    segs = _lib.debug_plan(msg, 0, MAX)
    assert [s["d"] for s in segs] == list(range(1, 21))
    prev_hi = -1
    r = (L + 1) % 64
    for s in segs:
        assert s["lo"] == prev_hi + 1 and _digits(s["lo"]) == _digits(s["hi"]) == s["d"]
        prev_hi = s["hi"]
        d, T = s["d"], r + s["d"]
        fb, p_end = (T - 1) // 64, (T - 1) % 64
        assert s["W1"] == p_end // 4
        assert s["straddle"] == (p_end % 4 == 0)
        assert s["trailer"] == (T + 9 > 64 and fb == 0)
        if s["kind"] == _lib.HM_KIND_TILED:
            V = s["V"]
            first = p_end - V + 1                    # first varying byte in block fb
            digit_start = r if fb == 0 else 0
            assert 5 <= V <= 8 and V <= d
            assert s["W1"] >= 1
            if s["lane3"]:  # lanes reach into W[W1-2]: only where two words give q < 5
                assert s["W1"] >= 2 and p_end % 4 in (0, 1) and V <= 7
                assert first >= digit_start and first >= 4 * (s["W1"] - 2)
                assert first < 4 * (s["W1"] - 1)
            else:
                assert first >= digit_start and first >= 4 * (s["W1"] - 1)
                # two words were enough, or the message prefix leaves no room
                assert V >= 7 or s["W1"] < 2 or first == digit_start
            assert (not s["trailer"]) or s["W1"] >= 13
        elif s["kind"] == _lib.HM_KIND_CHAINED:
            f = T - 64                              # digits in the final block
            q = s["V"] - f                          # lane digits, W15 (+ W14's last byte) of block 0
            assert fb == 1 and s["f"] == f and q == min(5, 64 - r)
            if f <= 4:                              # one table of 10^f rows
                assert 2 <= q <= 5 and s["fe"] == f
            else:                                   # table of the low fe digits, epochs above
                assert 3 <= q <= 5 and q + f <= 19 and s["fe"] == min(f, 7) and s["tch"] == 100
        else:
            assert s["kind"] == _lib.HM_KIND_GENERIC
    assert prev_hi == MAX


def test_planner_chained_epochs_where_cheaper():
    """Two-block tails with >= 5 final-block digits go chained (lanes in block
    0, K+W table of the low fe <= 6 final digits, epochs above) when the
    range spans enough lane values; a narrow range keeps the tiled layout,
    whose lanes vary the low digits."""
    m60 = b"x" * 60                                  # r = 61: 3 digits in block 0
    seg = _lib.debug_plan(m60, 10**9, 10**10 - 1)[0]  # d = 10: f = 7
    assert seg["kind"] == _lib.HM_KIND_CHAINED and (seg["f"], seg["fe"]) == (7, 7)
    narrow = _lib.debug_plan(m60, 5 * 10**9, 5 * 10**9 + 10**8)[0]
    assert narrow["kind"] == _lib.HM_KIND_TILED and narrow["W1"] == 1
    m58 = b"y" * 58                                  # r = 59: 5 digits in block 0
    seg = _lib.debug_plan(m58, 10**9, 10**10 - 1)[0]  # f = 5: one table, no epochs
    assert seg["kind"] == _lib.HM_KIND_CHAINED and (seg["f"], seg["fe"]) == (5, 5)
    assert seg["cost"] < 3300
    # cfg3's 120-B message keeps its f <= 4 tables (d = 8..10)
    assert all(s["kind"] == _lib.HM_KIND_CHAINED and s["f"] == s["fe"] <= 3
               for s in _lib.debug_plan(bytes(120), 10**7, 2**32 - 1))


def test_planner_bradfitz_2p32():
    segs = _lib.debug_plan(b"bradfitz", 0, 2**32 - 1)
    big = segs[-1]
    assert (big["d"], big["lo"], big["hi"], big["kind"], big["W1"], big["V"]) == \
        (10, 10**9, 2**32 - 1, _lib.HM_KIND_TILED, 4, 7)


def test_planner_force_generic():
    segs = _lib.debug_plan(b"bradfitz", 0, 10**12, force_generic=True)
    assert all(s["kind"] == _lib.HM_KIND_GENERIC for s in segs)


def test_planner_empty_and_single():
    assert _lib.debug_plan(b"x", 5, 4) == []
    s = _lib.debug_plan(b"x", MAX, MAX)
    assert len(s) == 1 and s[0]["lo"] == s[0]["hi"] == MAX


def test_planner_chained_epoch_cost_model():
    """The f >= 5 chained layout's modelled cost is 3275 SIMD cycles per 64
    nonces over the fraction of hashed nonces inside [lo, hi] (its lanes vary
    block-0 digits, stride 10^f nonces, so the 64-lane chunks at the range's
    ends carry out-of-range lanes); it is picked exactly when that beats the
    tiled layout's cost (plan.cpp consider_chained_epochs)."""
    import random
    rng = random.Random(4040)
    tiled_cost = {s["W1"]: s["cost"] for L in range(0, 45)
                  for s in _lib.debug_plan(b"x" * L, 10**9, 10**9 + 10**6)
                  if s["kind"] == _lib.HM_KIND_TILED and not s["trailer"]}
    n_chained = n_tiled = 0
    for _ in range(400):
        L = rng.choice([56, 57, 58, 59, 60, 120, 121, 122, 123, 124])
        r = (L + 1) % 64
        q = min(5, 64 - r)
        d = rng.randrange(64 - r + 5, 20)
        f = r + d - 64
        S, P = 10**f, 10**(q + f)
        span = rng.choice([rng.randrange(1, 64 * S), rng.randrange(64 * S, 64 * S * 40)])
        span = min(span, (10**d - 10**(d - 1)) // 2)
        lo = rng.randrange(10**(d - 1), 10**d - span)
        hi = lo + span - 1
        seg = _lib.debug_plan(b"x" * L, lo, hi)[0]
        tpt = -(-10**q // 64)
        chunks = (hi // P - lo // P) * tpt + (hi % P) // S // 64 - (lo % P) // S // 64 + 1
        eff = span / (chunks * 64 * S)
        if seg["kind"] == _lib.HM_KIND_CHAINED:
            n_chained += 1
            assert seg["f"] == f and abs(seg["cost"] - int(3275 / eff)) <= 1, (L, lo, hi)
            assert 3275 / eff < tiled_cost.get(seg["W1"], 6000 * 2)
        else:
            n_tiled += 1
            assert 3275 / eff >= seg["cost"] - 1 or q + f > 19, (L, lo, hi, seg)
    assert n_chained > 50 and n_tiled > 50, (n_chained, n_tiled)

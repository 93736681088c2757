"""The unchanged server's split/merge (server.go:165-205, 273-276) as modelled
for end-to-end expectations (SURVEY A-inv-7)."""
from distributed_bitcoinminer_amd import server_model as sm

MAX = (1 << 64) - 1


def test_load_balance_examples():
    assert sm.load_balance(0, 9999, 3) == [(0, 3334), (3334, 6667), (6667, 10000)]
    assert sm.load_balance(0, 2, 8) == [(0, 1), (1, 2), (2, 3)]
    ch = sm.load_balance(10**19, MAX - 1, 8)
    assert len(ch) == 8 and ch[-1] == (17390901064495857664, MAX)
    assert sm.load_balance(0, MAX, 4) == []  # totalLoad wraps to 0: never completes


def test_merge_arrival_order_and_seed():
    assert sm.merge_in_arrival_order([]) == (MAX, MAX)
    assert sm.merge_in_arrival_order([(MAX, 0)]) == (MAX, MAX)  # strict < never takes MAX
    assert sm.merge_in_arrival_order([(5, 9), (5, 1), (3, 7)]) == (3, 7)
    assert sm.merge_in_arrival_order([(5, 9), (5, 1)]) == (5, 9)  # ties: first arrival


def test_expected_client_result_config1(oracle_mod):
    def miner_scan(data, lower, upper):
        return oracle_mod.c_miner_eval(data, lower, upper, threads=4)
    # config 1 on one miner: server scans [0, 10^7+1]; client prints 356393768206 7645578
    assert sm.expected_client_result(b"bradfitz", 0, 9999, 3, miner_scan) == \
        (1419516646206828, 9898)
    # last chunk ends at 2^64-1 and scans nothing (A-inv-5 + A-inv-7)
    lo = MAX - 1 - 3000
    chunks = sm.load_balance(lo, MAX - 1, 3)
    assert chunks[-1][1] == MAX
    res = sm.expected_client_result(b"bradfitz", lo, MAX - 1, 3, miner_scan)
    assert res == oracle_mod.c_scan(b"bradfitz", lo, chunks[-1][0], threads=4)

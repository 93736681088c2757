"""CPU oracle for the min-hash nonce scan -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  The product (distributed_bitcoinminer_amd + libhipminer.so)
never imports, links or falls back to it.
"""

"""CPU oracle package — TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).

Parity is pinned against fixtures generated from the reference itself
(tests/golden/make_goldens.py); see cvae_oracle.py for the citations.
"""

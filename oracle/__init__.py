"""oracle/ -- TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference algorithm on the hot path (numpy, float32 arithmetic in the
reference's op order). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker / the timed CPU baseline -- never as a product
path. Parity pinning: tests/test_oracle_golden.py checks every function here against golden
fixtures captured from the reference itself (tests/golden/make_golden.py).
"""
from .dmip_oracle import *  # noqa: F401,F403

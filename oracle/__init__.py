"""CPU restatement of Pyrope's C# ANN engine -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / the timed CPU baseline.  The product
path (pyrope_amd, libpyrope_hip.so) never imports it.
"""
from .oracle import *  # noqa: F401,F403

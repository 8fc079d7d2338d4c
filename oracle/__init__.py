"""CPU restatement of the consensusClust hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package.  The product (consensusclustr_amd) never does.
PARITY UNPINNED: see ccg_oracle.c header and DESIGN.md section "Oracle".
"""
from .oracle import *  # noqa: F401,F403

"""oracle — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference hot path (C: walk.c; numpy/torch-CPU:
cpu_ref.py). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may import it, as the checker or the timed CPU baseline. The product
package recbole_amd never imports it (tests/test_boundary.py enforces this).
"""

"""CPU oracle for the DISORT flux path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py (cpu_baseline) may import
this package.  The product (pyharp_amd) never does.
"""

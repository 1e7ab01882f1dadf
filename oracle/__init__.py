"""CPU oracle — TEST INFRASTRUCTURE ONLY (see oracle.py / gf_oracle.c headers).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package; the product (hummingbird_amd / libhbec.so) never does.
"""

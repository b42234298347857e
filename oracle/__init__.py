"""oracle/ -- TEST INFRASTRUCTURE ONLY.

CPU restatement of DeepReadMapper's query hot path (see drm_oracle.h for citations) plus loaders
for the reference-built checker (oracle/_ref). Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this package; the product path (deepreadmapper_amd) never does.
"""

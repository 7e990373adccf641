"""ORACLE package -- test infrastructure only (see oracle/vdp_oracle.py header).

CPU restatements of the reference hot path used as the parity checker by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg.  Never imported by vent_analysis_amd.
"""

"""Import-compatible stand-in for the reference's ``deepspeed/smt`` package.

``deepspeed/fine_tune.py:39-40`` imports ``smt.smt`` and ``smt.smt_helper``; with this repository's
root on ``sys.path`` those imports resolve here and bind the MI355X implementation
(:mod:`sparse_matrix_tuning_amd.smt`). Unlike the reference (smt.py:20, smt_helper.py:12), importing
does not initialise a process group.
"""

"""Import-compatible stand-ins for the reference's ``smt.smt`` and ``smt.smt_helper``
(deepspeed/fine_tune.py:39-40)."""

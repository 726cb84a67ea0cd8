"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

A plain restatement (numpy / pure Python / C) of the reference algorithms on
the MI355X hot path, each function citing the reference file:line it follows
(paths relative to the mcx/AgileRL checkout).  It exists to CHECK the HIP
product path and to provide the timed CPU baseline in ``bench.py``.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import, call, link or execute anything under
``oracle/``.  The product package ``agilerl_amd`` never imports it and has no
CPU fallback: without the HIP library it raises.

Pinning: every restatement here is checked against golden vectors produced by
the reference's own code (``tests/golden/gen_golden.py`` executes the
reference source files in place and records inputs/outputs) and against the
reference's own known-answer tests (``tests/test_components/
test_segment_tree.py``, ``test_replay_buffer.py:901-1039`` upstream), see
``tests/test_oracle_golden.py``.
"""

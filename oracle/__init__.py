"""CPU oracle for the PH hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import this package, and only as the checker / CPU baseline.
The product path (``mpi-sppy-1_amd/mpisppy_amd``) never imports it and has no
CPU fallback.

Contents (each function cites the reference file:line it restates; paths are
relative to the reference repository ulysse-n/mpi-sppy-1):

* ``models``  -- restatement of the farmer (examples/farmer/farmer.py:25-224) and
  aircond (mpisppy/tests/examples/aircond.py:37-330) scenario models as explicit
  LP/QP row lists, including the seeded RNG streams.
* ``lpqp``    -- exact per-scenario solvers standing in for the external
  LP/QP solver the reference reaches through Pyomo's SolverFactory
  (spopt.py:85-223): a closed-form farmer prox solver, a dense Mehrotra
  interior-point QP solver with active-set polish, and scipy's HiGHS for LPs.
* ``ph``      -- restatement of PHBase (phbase.py:27-107, 293-343, 758-979),
  SPOpt.Ebound / Eobjective (spopt.py:310-391) and the rank partition
  (sputils.py:774-840).

Pinning: the restatement reproduces the reference's own fixtures
mpisppy/tests/examples/w_test_data/{w_file,xbar_file}.csv (test_w_writer.py:85-117),
the trivial bound of test_aph.py:230-253 and the EF optimum of test_sc.py:30-38;
see tests/test_oracle_golden.py.
"""

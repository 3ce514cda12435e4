"""CPU oracle for the batched condensed-QP MPC hot path -- TEST INFRASTRUCTURE ONLY.

This package is the *checker*, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import,
call, link or execute anything under ``oracle/``.  The product path
(``model_predictive_control_amd``) never imports it and fails loudly when its
HIP library is missing.

Contents (each function cites the reference file:line it restates):

* ``oracle.session1``  -- ``session_1/FHC.py``, ``session_1/LinearSystem.py`` and
  ``session_1/session1_sol.py`` in plain NumPy (Riccati recursion, closed-loop
  simulation, prediction).  Pinned bit-for-bit-ish (<=1e-12) against golden
  vectors captured from the importable reference (``tests/golden/``).
* ``oracle.condense`` -- the single-shooting condensing of
  ``session_4/main.py:86-106`` / ``session_4/session4_sol.py:195-204`` written
  out as explicit matrices (Phi, Gamma, H, F, f, state-constraint rows).
  Pinned by the closed-form Riccati <-> condensed equivalence.
* ``oracle.qp``       -- exact fp64 active-set solvers for the box QP and the
  polytope QP, with KKT certificates; SciPy BVLS is used as an independent
  cross-check for box QPs.  The reference solves these with CasADi/IPOPT
  (``session_4/main.py:38-39,115-116``), which is not installed here: parity
  against IPOPT is *unpinned*; optimality is certified by KKT residuals
  instead (a strictly convex QP has a unique minimiser).
* ``oracle.bicycle``  -- kinematic bicycle ODE + FE/RK4 discretisation
  (``session_4/main.py:132-147``).  ``rcracers.KinematicBicycle`` is absent
  from the container, so the ODE itself is *parity unpinned*.
* ``oracle/c/``        -- a C restatement of condense + box-QP used only as the
  CPU baseline in ``bench.py`` (``cpu_baseline.kind = "port"``).
"""

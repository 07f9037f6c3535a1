"""CPU oracle for the MuZero-Go self-play hot path -- TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU, the reference algorithm that the MI355X
engine (``muzero-go_amd/``) implements in HIP.  It exists to *check* the
engine, never to run in its place:

* only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
  ``cpu_baseline`` leg may import it;
* the product (``mzgo``) never imports it and has no CPU fallback.

Modules and what they restate (all citations into the reference snapshot):

=================  ===========================================================
``npsum``          numpy 2.2.6 pairwise float reduction order (the f32/f64
                   ``policy.sum()`` calls at self_play.py:160,170,211,378)
``rng``            the counter-based RNG the engine uses in place of CPython
                   ``random.choice`` / numpy ``RandomState`` (hook streams)
``weights``        deterministic PyTorch-default-scaled weight generator
``net``            ``MuZeroNet`` and its three networks, self_play.py:63-128
``gogame``         GymGo rules (``gogame.py`` / ``state_utils.py``) used by
                   self_play.py:14,152,363,479,502,544 -- see "parity" below
``goenv``          GymGo ``GoEnv`` (reset/step/winner/reward)
``mcts``           ``MCTSNode`` / ``MCTS`` / ``apply_dirichlet_noise``,
                   self_play.py:36-39,131-343
``selfplay``       ``MuZeroAgent.select_action``, ``GameHistory``,
                   ``run_self_play_game`` and the pickle batch writer,
                   self_play.py:347-596
``make_golden``    fixture generator: imports the reference itself (in the
                   build container only) and writes ``tests/golden/``
=================  ===========================================================

Parity status
-------------
* net / MCTS / agent / game record: **pinned** -- ``tests/golden/`` holds
  vectors produced by importing the reference ``self_play.py`` in the build
  container (``oracle/make_golden.py``), and ``tests/test_oracle_golden.py``
  checks this restatement against them bit-for-bit (MCTS, records) or at
  fp32 tolerance (net).
* board rules (GymGo): **parity unpinned**.  GymGo (``huangeddie/GymGo``,
  un-vendored submodule, installed by unpinned ``git clone``; README.md:7-13)
  is absent from the reference snapshot and from this image, and the
  reference holds no test or fixture for board results.  ``gogame`` restates
  upstream master's published algorithm with the same ``scipy.ndimage``
  primitives and is pinned only by hand-written known-answer positions
  (``tests/test_oracle_gogame.py``).
"""

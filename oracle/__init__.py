"""CPU oracle for the asrx hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package, and
only as the checker / the timed CPU baseline, never as the measured or shipped path.

What it is: an op-for-op CPU restatement of the reference's live forward path (sine2pi/ASR-model
model.py + essentials.py, cited file:line in each function), with the reference's randomness
(gumbel noise, dropout masks) taken as explicit, keyed inputs (oracle/noise.py).

Pinning status: PARITY UNPINNED.  The reference ships no tests, fixtures or golden vectors, its
third-party deps (torchaudio, tensordict, pyworld) are absent, and importing/executing the
reference was denied in this pipeline.  The restatement is checked by
known-answer tests (tests/test_oracle.py) and line-by-line review against the cited source.
"""

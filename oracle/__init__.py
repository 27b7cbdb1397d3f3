"""Test infrastructure only: CPU oracle for the Genie-TTS hot path.

Nothing in the product package (`genie_tts_amd`) may import from here; only
`tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg use it,
and only as the checker / CPU baseline, never as the measured or shipped path.
"""

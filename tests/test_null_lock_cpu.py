"""ofdmProcessor::run's null search locking onto the frame period after a sync loss, pinned
on the oracle (the reference's algorithm restated, ofdm-processor.cpp:272-327): the stream
bench.py's four-rank rehearsal found (tests/null_lock.py).  CPU only;
the GPU pipeline's equality on the same stream is test_gpu_pipeline_oracle.py's
test_pipeline_null_lock_like_reference."""
import numpy as np

import null_lock as nl
import oracle_py as orc


def test_null_search_locks_onto_frame_period_like_reference():
    _, x = nl.stream()
    n_samples = len(x) // 2
    n, info, _ = orc.ofdm_run(x, nl.FRAMES, threshold=3, method=1)
    # the jammed frame is the last one decoded: 124 frames of clean signal follow
    assert n == 229 and info[-1].window_start == nl.LAST_WINDOW
    after = nl.LAST_WINDOW + nl.TF
    found, _, _, pos = orc.null_scan(x[2 * after:], n_samples - after, scan=False)
    assert not found and pos == n_samples - after
    # the stream is fine: the same search begun after the interferer ends finds a null
    assert orc.null_scan(x[2 * 45_400_000:], 2 * nl.TF, scan=False)[0] == 1
    # every attempt: a dip one frame after the last, its end not seen within T_null + 50
    tr = nl.trace_null_search(x, after, 3)
    assert all(d is not None and e is None for d, e, _ in tr), tr
    dips = [d for d, _, _ in tr]
    assert all(abs(dips[k + 1] - dips[k] - nl.TF) < 50 for k in range(len(dips) - 1)), dips
    # sLevel has climbed to most of the envelope's mean by the time the dip comes
    z = x[2 * 45_400_000:2 * 46_400_000].reshape(-1, 2)
    mean = float(np.mean(np.abs(z[:, 0]) + np.abs(z[:, 1])))
    assert all(s > 0.8 * mean for _, _, s in tr[1:]), (tr, mean)

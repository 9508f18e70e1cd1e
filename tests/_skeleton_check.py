"""Child-process check (run with PYTHONHASHSEED=0, the seed the reference ran
under in tests/golden/make_callers_golden.py): the mirrors'
SkeletonBuilder._predict_skeleton per side and select_sequence_length_with_
jaccard on the filter's output equal the reference's own results
(callers.json.gz "skeleton").  Explanation lists follow Python set order in
the reference and in the mirror alike, so the hash seed must match.

usage: python tests/_skeleton_check.py TEST_ID [cpu|gpu|device]
TEST INFRASTRUCTURE."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]


def main():
    tc, mode = sys.argv[1], sys.argv[2]
    assert os.environ.get("PYTHONHASHSEED") == "0", "run with PYTHONHASHSEED=0"
    import pytest

    import _callers_checks as C
    from conftest import load_golden

    engine = None
    if mode == "device":
        from spectrseqtools_amd import _native

        engine = _native.get_engine(0)
    elif mode == "cpu":
        import _fake_engine

        _fake_engine.install(pytest.MonkeyPatch())
    else:
        from spectrseqtools_amd import _native

        engine = _native.get_engine(0)
    rec = load_golden("callers.json.gz")[tc]
    rec["_tc"] = tc
    dp = C.make_dp(rec["ctx"], engine=engine)
    if mode == "device":  # the device-resident pipeline (k_skel_walk)
        sk = C.check_skeleton_device_vs_reference(rec, dp)
        print(f"skeleton ok {tc} device launches={sk.launches} requeries={sk.requeries}")
        return
    classified = C.check_classify(rec, dp)
    frags, expl = C.check_filter(rec, dp)
    C.check_skeleton_vs_reference(rec, dp, frags, expl)
    # Predictor.predict up to the skeleton-based reduction, from a fresh table
    C.check_predict_skeleton_stage(rec, C.make_dp(rec["ctx"], engine=engine), classified)
    print(f"skeleton ok {tc}")


if __name__ == "__main__":
    main()

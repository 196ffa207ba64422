"""calculate_metrics (code/utils.py:38-55): micro / macro P/R/F1 and the per-class sensitivity /
specificity table, checked against sklearn's one-vs-rest recall and a direct confusion count."""
import numpy as np
import pytest

from endossl.utils import AttrDict, calculate_metrics


def _cfg(c):
    return AttrDict(MODEL=AttrDict(NUM_CLASSES=c))


def test_sen_spec_matches_confusion_counts():
    from sklearn.metrics import recall_score
    rng = np.random.default_rng(0)
    C = 23
    target = rng.integers(0, C, 500)
    pred = np.where(rng.random(500) < 0.6, target, rng.integers(0, C, 500))
    m = calculate_metrics(list(pred), list(target), _cfg(C))
    df = m["sen/spec"]
    assert list(df.columns) == ["class", "sensitivity", "specificity"]
    assert list(df["class"]) == list(range(C))
    for c in range(C):
        t, p = target == c, pred == c
        tp, fn = int((t & p).sum()), int((t & ~p).sum())
        tn, fp = int((~t & ~p).sum()), int((~t & p).sum())
        sen = tp / (tp + fn) if tp + fn else 0.0
        spec = tn / (tn + fp) if tn + fp else 0.0
        assert df["sensitivity"][c] == pytest.approx(sen, abs=1e-12)
        assert df["specificity"][c] == pytest.approx(spec, abs=1e-12)
        # the reference's own call: recall of the positive / negative label of the one-vs-rest problem
        assert df["sensitivity"][c] == pytest.approx(recall_score(t, p, pos_label=True, zero_division=0))
        assert df["specificity"][c] == pytest.approx(recall_score(t, p, pos_label=False, zero_division=0))
    # macro recall is the mean per-class sensitivity over the classes present
    present = np.unique(np.concatenate([target, pred]))
    assert m["macro/recall"] == pytest.approx(df["sensitivity"][present].mean())


def test_sen_spec_absent_class_and_no_config():
    target = np.array([0, 1, 1, 2])
    pred = np.array([0, 1, 2, 2])
    m = calculate_metrics(pred, target, _cfg(5))  # classes 3, 4 never occur
    df = m["sen/spec"]
    assert len(df) == 5
    assert df["sensitivity"][3] == 0.0 and df["specificity"][3] == 1.0
    assert df["sensitivity"][1] == 0.5 and df["specificity"][2] == pytest.approx(2 / 3)
    m2 = calculate_metrics(pred, target)  # config None: max label + 1 classes
    assert len(m2["sen/spec"]) == 3

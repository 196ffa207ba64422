"""Host-side helpers mirroring code/utils.py (AttrDict :16-19, AverageMeter :21-36,
calculate_metrics :38-55, get_config :128-134, count_parameters :154-155)."""
import numpy as np
import yaml
from yaml.loader import SafeLoader


class AttrDict(dict):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.__dict__ = self


class AverageMeter:
    """Computes and stores the average and current value (code/utils.py:21-36)."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.val = 0
        self.avg = 0
        self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count


# Keys the SSL hot path dereferences (SURVEY.md §5 "Config / flags").  Several reference configs
# omit some of them (PRE_TRAIN_RESUME, IS_FREEZE, SAVE_CP) and crash at code/learn.py:79; the
# loader fills these defaults instead.
DEFAULTS = {
    "DATA": {"BATCH_SIZE": 64, "MU": 7, "IMG_SIZE": 224, "TARGET_NAME": "target", "NUM_WORKERS": 2},
    "MODEL": {"NAME": "vit_small_patch16_224", "NUM_CLASSES": 23, "TYPE_SEMI": "FixMatch", "LOW_DIM": 64,
              "MARGIN": "None", "PRE_TRAIN_PATH": "None", "PRE_TRAIN_RESUME": "None", "PRE_TRAIN": False,
              "IS_TRIPLET": False},
    "TRAIN": {"IS_SSL": True, "IS_FREEZE": False, "USE_EMA": True, "EMA_DECAY": 0.999, "BASE_LR": 1e-3,
              "WARMUP_LR": 5e-4, "WARMUP_EPOCHS": 0, "DECAY_EPOCHS": 10, "LR_DECAY": 0.8, "SCH_NAME": "step",
              "EVAL_STEP": 256, "EVAL_STEP_SUP": 0, "CLS_WEIGHT": True, "THRES": 0.95, "T": 1.0,
              "LAMBDA_U": 1.0, "LAMBDA_C": 1.0, "EPOCHS": 150, "FREQ_EVAL": 5, "SAVE_CP": ".",
              "OPT_NAME": "Adam"},
}


def with_defaults(config):
    for sec, vals in DEFAULTS.items():
        if sec not in config:
            config[sec] = AttrDict()
        for k, v in vals.items():
            if k not in config[sec]:
                config[sec][k] = v
    return config


def get_config(config_file, fill_defaults=True):
    """YAML -> AttrDict of AttrDicts (code/utils.py:128-134), SafeLoader only."""
    with open(config_file) as f:
        config = yaml.load(f, Loader=SafeLoader)
    config = AttrDict(config)
    for k1 in config.keys():
        config[k1] = AttrDict(config[k1])
    return with_defaults(config) if fill_defaults else config


def count_parameters(model):
    return sum(p.numel() for p in model.parameters() if p.requires_grad)


def sen_spec(pred, target, num_classes):
    """Per-class sensitivity / specificity (code/utils.py:41-46): class l's one-vs-rest problem
    (target == l, pred == l) through precision_recall_fscore_support(average=None); the recall of
    the positive label is the sensitivity, that of the negative label the specificity.  labels=
    [False, True] is passed explicitly: the reference's call infers the labels, so a class absent
    from both target and pred yields one label and its recall[1] raises IndexError; here that class
    reads sensitivity 0, specificity 1."""
    import pandas as pd
    from sklearn.metrics import precision_recall_fscore_support
    pred, target = np.asarray(pred), np.asarray(target)
    rows = []
    for c in range(num_classes):
        _, recall, _, _ = precision_recall_fscore_support(target == c, pred == c, labels=[False, True], average=None,
                                                          zero_division=0)
        rows.append([c, recall[1], recall[0]])
    return pd.DataFrame(rows, columns=["class", "sensitivity", "specificity"])


def calculate_metrics(pred, target, config=None):
    """Micro/macro P/R/F1 and the per-class sensitivity / specificity table (code/utils.py:38-55);
    host-side, evaluation only.  config.MODEL.NUM_CLASSES sets the table's classes (config None:
    max label + 1)."""
    from sklearn.metrics import f1_score, precision_score, recall_score
    pred, target = np.asarray(pred), np.asarray(target)
    try:
        ncls = int(config.MODEL.NUM_CLASSES)
    except (AttributeError, KeyError, TypeError):
        ncls = int(max(pred.max(initial=-1), target.max(initial=-1))) + 1
    return {
        "micro/precision": precision_score(target, pred, average="micro", zero_division=0),
        "micro/recall": recall_score(target, pred, average="micro", zero_division=0),
        "micro/f1": f1_score(target, pred, average="micro", zero_division=0),
        "macro/precision": precision_score(target, pred, average="macro", zero_division=0),
        "macro/recall": recall_score(target, pred, average="macro", zero_division=0),
        "macro/f1": f1_score(target, pred, average="macro", zero_division=0),
        "sen/spec": sen_spec(pred, target, ncls),
    }


def balanced_class_weights(labels):
    """sklearn class_weight='balanced' = n / (k * bincount) over the labeled targets
    (code/fixmatch.py:61-66; classes passed as an ndarray, which sklearn>=1.x requires)."""
    from sklearn.utils import class_weight
    y = np.asarray(list(labels))
    return class_weight.compute_class_weight(class_weight="balanced", classes=np.unique(y), y=y).astype(np.float32)

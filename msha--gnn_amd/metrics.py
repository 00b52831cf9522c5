"""Host-side evaluation helpers train.py reaches through ``from model import *``
(model.py:66-92).  Not part of the GPU path: plain sklearn on host arrays."""
import numpy as np


def calculate_auc(y_pred, y_true):
    """Macro one-vs-rest AUC over the classes present in y_true."""
    from sklearn.metrics import roc_auc_score
    from sklearn.preprocessing import label_binarize

    classes = np.unique(y_true)
    yb = label_binarize(y_true, classes=classes)
    return float(np.mean([roc_auc_score(yb[:, c], np.asarray(y_pred)[:, c])
                          for c in range(yb.shape[1])]))


def calculate_accuracy(predicted_labels, true_labels):
    from sklearn.metrics import accuracy_score

    return accuracy_score(true_labels, predicted_labels)


def calculate_precision_recall(predicted_labels, true_labels, model):
    from sklearn.metrics import precision_score, recall_score

    return (precision_score(true_labels, predicted_labels, average=model, zero_division=1),
            recall_score(true_labels, predicted_labels, average=model, zero_division=1))

"""Restatement of the Clip facade math (src/clip.rs:79-185) — TEST INFRASTRUCTURE.

compare:      dot(v, t).mul_add(scale, bias)                       (:81-90)
classify:     logits = (T @ v) * scale + bias; sigmoid | softmax; sort desc  (:94-132)
rank_images:  logits = (V @ t) * scale + bias; same                 (:136-170)
softmax:      max-subtracted exp / sum                              (:174-179)
sigmoid:      1 / (1 + exp(-l))                                     (:183-185)
scale / bias default to 1.0 / 0.0; activation defaults to "softmax".
"""
import numpy as np


def softmax(logits):
    x = np.asarray(logits, np.float64)
    e = np.exp(x - x.max())
    return e / e.sum()


def sigmoid(l):
    return 1.0 / (1.0 + np.exp(-np.asarray(l, np.float64)))


def probs(logits, activation):
    return sigmoid(logits) if activation == "sigmoid" else softmax(logits)


def classify(img_emb, text_embs, labels, scale=1.0, bias=0.0, activation="softmax"):
    logits = np.asarray(text_embs, np.float64) @ np.asarray(img_emb, np.float64) * scale + bias
    p = probs(logits, activation)
    order = sorted(range(len(labels)), key=lambda i: -p[i])
    return [(labels[i], float(p[i])) for i in order]


def rank_images(img_embs, text_emb, scale=1.0, bias=0.0, activation="softmax"):
    logits = np.asarray(img_embs, np.float64) @ np.asarray(text_emb, np.float64) * scale + bias
    p = probs(logits, activation)
    order = sorted(range(len(p)), key=lambda i: -p[i])
    return [(i, float(p[i])) for i in order]


def compare(img_emb, text_emb, scale=1.0, bias=0.0):
    return float(np.dot(np.asarray(img_emb, np.float64), np.asarray(text_emb, np.float64)) * scale + bias)

#!/usr/bin/env python3
"""Independent optimum pin for config C1: solve the same hinge-loss SVM with
scikit-learn's liblinear (dual CD, no bias, C = 1/(lambda*n)) and record the
primal objective in the reference's form (OptUtils.scala:73-75):
    P(w) = mean_i max(1 - y_i x_i.w, 0) + lambda/2 ||w||^2.
Test infrastructure only; writes tests/golden/c1_liblinear.json."""
import json, os, sys
import numpy as np
from scipy.sparse import csr_matrix
from sklearn.svm import LinearSVC

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle  # noqa: E402

d = oracle.Data.load_libsvm(os.path.join(HERE, "data", "small_train.dat"), 4, 9947)
X = csr_matrix((d.val, d.col, d.row_ptr), shape=(d.n, d.d))
lam = 1e-3
clf = LinearSVC(loss="hinge", dual=True, C=1.0 / (lam * d.n), fit_intercept=False, tol=1e-12, max_iter=2000000)
clf.fit(X, d.y)
w = clf.coef_.ravel()
P = float(np.mean(np.maximum(1 - d.y * (X @ w), 0)) + 0.5 * lam * (w @ w))
json.dump({"lambda": lam, "primal_opt": P, "sklearn_tol": 1e-12,
           "train_err": int(np.sum(d.y * (X @ w) <= 0))}, open(os.path.join(HERE, "c1_liblinear.json"), "w"), indent=1)
print(P)

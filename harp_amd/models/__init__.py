"""Applications (Harp L6): K-means, MF-SGD, CCD, LDA, PCA/Cov/MOM, regressions, ..."""

"""visreps_amd — MI355X-native RSA eval hot path of yashsmehta/visreps.

feature extraction -> N x N Pearson RDM (fp32 MFMA Gram) -> sorted-triangle midrank
Spearman -> bootstrapped Spearman RSA, behind the reference's visreps.analysis /
visreps.evals / visreps.run API. See DESIGN.md.
"""
__version__ = "0.1.0"

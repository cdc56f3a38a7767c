"""MI355X-native TencentGR sequence-recommender training path (grk).

Drop-in for the hot path of Puiching-Memory/Tencent_Recommendation_2025's
``model/BaseLine`` training script: ``model.BaselineModel`` and
``dataset.MyDataset`` keep the reference surface; device work runs in
hand-written gfx950 HIP kernels (libgrk.so, C ABI in include/grk.h).
"""
__version__ = '0.1.0'

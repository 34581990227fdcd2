from recbole_amd.model.context_aware_recommender.deepfm import DeepFM

__all__ = ['DeepFM']

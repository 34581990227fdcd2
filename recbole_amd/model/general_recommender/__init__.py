from recbole_amd.model.general_recommender.bpr import BPR

__all__ = ['BPR']

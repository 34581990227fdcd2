from recbole_amd.model.sequential_recommender.sasrec import SASRec

__all__ = ['SASRec']

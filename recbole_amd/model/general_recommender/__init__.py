from recbole_amd.model.general_recommender.bpr import BPR
from recbole_amd.model.general_recommender.lightgcn import LightGCN

__all__ = ['BPR', 'LightGCN']

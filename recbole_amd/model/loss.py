"""Loss modules (mirror of recbole/model/loss.py:23-84). The BPR training
path does not call BPRLoss.forward: BPR.calculate_loss runs the fused K3
kernel (csrc/bpr.hip) that computes this loss and its gradient in one pass.
These modules stay for API compatibility with user code."""
import torch
import torch.nn as nn


class BPRLoss(nn.Module):

    def __init__(self, gamma=1e-10):
        super().__init__()
        self.gamma = gamma

    def forward(self, pos_score, neg_score):
        return -torch.log(self.gamma + torch.sigmoid(pos_score - neg_score)).mean()


class EmbLoss(nn.Module):

    def __init__(self, norm=2):
        super().__init__()
        self.norm = norm

    def forward(self, *embeddings):
        emb_loss = torch.zeros(1).to(embeddings[-1].device)
        for e in embeddings:
            emb_loss += torch.norm(e, p=self.norm)
        emb_loss /= embeddings[-1].shape[0]
        return emb_loss

"""Kubernetes contract (annotations, resource names), API client and in-memory fake apiserver."""
from .annotations import ANN_ASSIGNED, ANN_ASSUME_TIME, ANN_GPU_ID_ALIAS, ANN_GROUP, Contract, PodAssignment
from .api import ApiError, Conflict, KubeAPI, NotFound, RestKubeAPI
from .fake import FakeAPIServer, serve_http

__all__ = [
    "ANN_ASSIGNED", "ANN_ASSUME_TIME", "ANN_GPU_ID_ALIAS", "ANN_GROUP", "Contract", "PodAssignment",
    "ApiError", "Conflict", "KubeAPI", "NotFound", "RestKubeAPI", "FakeAPIServer", "serve_http",
]

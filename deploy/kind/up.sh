#!/usr/bin/env bash
# BASELINE config 1: kind + 2 fake GPUs; the pod must reach Succeeded with GTK_GPU_GROUP set.
set -euo pipefail
cd "$(dirname "$0")"
kind create cluster --name gpu-topology --config kind-config.yaml
kind load docker-image --name gpu-topology rocm/gpu-topology-k8s:latest
kubectl apply -f gpu-topology-kind.yaml
kubectl -n kube-system rollout status ds/amd-gpu-topology-device-plugin --timeout=180s
kubectl -n kube-system rollout status ds/gpu-topology-scheduler-extender --timeout=180s
kubectl apply -f pod-1gpu.yaml
kubectl wait --for=jsonpath='{.status.phase}'=Succeeded pod/gpu-topology-smoke --timeout=180s
kubectl get pod gpu-topology-smoke -o jsonpath='{.metadata.annotations}'; echo
kubectl logs gpu-topology-smoke

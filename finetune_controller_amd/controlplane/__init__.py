"""Control plane: FastAPI API, job store, object store, Kubeflow/Kueue submission, reconciler, log streaming."""

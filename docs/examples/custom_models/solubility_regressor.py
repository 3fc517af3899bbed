"""Walkthrough A (docs/models.md): a spec for YOUR OWN training image.

A small regression model (molecular solubility from a CSV of numeric descriptors) trained by the
script ``docs/examples/train_regressor.py``, which the image would carry as ``/app/train_regressor.py``.
Drop this file into the directory named by ``CUSTOM_MODELS_DIR`` and restart the API: the model
appears in ``GET /api/v1/models`` with a form generated from ``SolubilityArguments``.

Self-check (no cluster needed)::

    python docs/examples/custom_models/solubility_regressor.py
"""
from pydantic import Field

from finetune_controller_amd.controlplane.spec.finetuning import (BaseFineTuneModel, TrainingArguments,
                                                                  TrainingDataset, TrainingFramework,
                                                                  TrainingResources, TrainingTask)


class SolubilityArguments(TrainingArguments):
    """Training flags: the JSON schema of this class is the UI form; user JSON is validated against it."""

    epochs: int = Field(default=20, ge=1, le=1000, description="Passes over the dataset")
    lr: float = Field(default=0.05, gt=0, description="Learning rate (full-batch gradient descent)")
    l2: float = Field(default=1e-4, ge=0, description="L2 weight decay")
    target_column: str = Field(default="solubility", description="CSV column to predict")


class SolubilityRegressor(BaseFineTuneModel):
    name: str = "Solubility-Regressor"
    inference_name: str | None = "Solubility"
    description: str = "Linear solubility regressor on molecular descriptors (CPU job, walkthrough A)"
    project_url: str = "https://example.org/solubility"
    image: str = "registry.example.org/ftc/solubility-trainer:0.1"
    command: list[str] = ["/bin/bash", "-c", "python /app/train_regressor.py"]
    framework: TrainingFramework = TrainingFramework.PYTORCH
    task: TrainingTask = TrainingTask.REGRESSION
    dataset_info: TrainingDataset = TrainingDataset(
        description="CSV with numeric descriptor columns and a 'solubility' column", dataset_required=True)
    resources: TrainingResources = TrainingResources(requests={"cpu": 2, "memory": "2Gi"},
                                                     limits={"cpu": 4, "memory": "4Gi"})
    # CPU job: the reference's convention -- a default below ge=1 is not validated and means "no GPU"
    accelerator_count: int = Field(default=0, ge=1, description="GPUs per worker (0: CPU job)")
    promotion_path: str = Field(default="molecules/solubility/linear", description="s3 promotion prefix")
    training_arguments: SolubilityArguments = SolubilityArguments()

    def run_cmd(self) -> list[str]:
        t = self.training_arguments
        return self.append_args([f"--epochs={t.epochs}", f"--lr={t.lr}", f"--l2={t.l2}",
                                 f"--target-column={t.target_column}"])


if __name__ == "__main__":  # self-check: the form, a validated instance and the container command
    import json

    print(json.dumps(SolubilityArguments.model_json_schema()["properties"], indent=1))
    m = SolubilityRegressor.model_validate(SolubilityRegressor(training_arguments={"epochs": 5, "lr": 0.1}))
    print(m.run_cmd())

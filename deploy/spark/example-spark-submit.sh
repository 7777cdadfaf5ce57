#!/bin/bash
# Spark-on-K8s img2dataset job (spark/example-spark-submit.sh of the reference):
# driver + executors on CPU nodes via cpu-pod-template.yaml, output on spark-pvc.
NAMESPACE=$(kubectl config view --minify -o jsonpath='{..namespace}')
echo "Using the namespace: $NAMESPACE"
IMAGE=${IMAGE:-ghcr.io/kubernetes-cloud-amd/kca:rocm7.2-gfx950}
K8S_API=${K8S_API:-https://kubernetes.default.svc}

$SPARK_HOME/bin/spark-submit \
    --master "k8s://$K8S_API" \
    --deploy-mode cluster \
    --name download-mscoco-16-64 \
    --conf spark.driver.cores=16 \
    --conf spark.kubernetes.driver.limit.cores=16 \
    --conf spark.driver.memory="64G" \
    --conf spark.executor.cores=16 \
    --conf spark.kubernetes.executor.limit.cores=16 \
    --conf spark.executor.memory="64G" \
    --conf spark.executor.instances=1 \
    --conf spark.kubernetes.driver.container.image="$IMAGE" \
    --conf spark.kubernetes.executor.container.image="$IMAGE" \
    --conf spark.kubernetes.driver.podTemplateFile=./cpu-pod-template.yaml \
    --conf spark.kubernetes.executor.podTemplateFile=./cpu-pod-template.yaml \
    --conf spark.kubernetes.namespace="$NAMESPACE" \
    --conf spark.kubernetes.authenticate.driver.serviceAccountName=spark-sa \
    local:///app/kubernetes_cloud_amd/data/img2dataset.py --output /mnt/pvc/mscoco -t 2048

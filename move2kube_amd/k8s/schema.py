"""Go ``encoding/json`` marshalling rules for the Kubernetes/OpenShift/Knative/
Tekton types the framework emits.

The reference writes every object as ``json.Marshal(typedObject)`` -> YAML
(``internal/transformer/transformer.go:162-204``).  Which empty fields appear
is decided by the Go struct tags: non-pointer structs are always emitted
(``resources: {}``, ``status: {}``, ``strategy: {}``), a zero ``metav1.Time``
marshals as ``null`` (``creationTimestamp: null``), fields without
``omitempty`` emit their zero value (``containerPort``, ``replicas`` of a
DeploymentConfig, ``currentNumberScheduled`` of a DaemonSet ...), and unknown
fields are dropped by the typed decode.  :func:`marshal` applies exactly those
rules to JSON-shaped dicts using the struct tables below.

Field DSL: ``"jsonName:type[,o]"`` where ``,o`` marks ``omitempty`` and type is
one of ``string int bool map any Time Quantity IntOrString bytes ArrayOrString``,
a struct name, ``*T`` (pointer), ``[]T`` (slice), ``map:T`` (map of T) or
``inline:T`` (embedded struct).
"""

import _thread

_STRUCTS = {}  # struct name -> its field DSL string (parsed on use: _fields)
_parsed = {}


def _def(name, spec):
    _STRUCTS[name] = spec


def _fields(name):
    """[(json name, field type, omitempty)] of a struct.  Parsed when first
    needed: a CLI run hands the strings to the native marshaller, which parses
    them itself, and only the Python fallback and the checks need tuples."""
    fields = _parsed.get(name)
    if fields is None:
        fields = []
        for item in _STRUCTS[name].split():
            o = item.endswith(",o")
            if o:
                item = item[:-2]
            jname, typ = item.split(":", 1)
            fields.append((jname, typ, o))
        _parsed[name] = fields
    return fields


# -- meta --------------------------------------------------------------------
_def("TypeMeta", "kind:string,o apiVersion:string,o")
_def("ObjectMeta", "name:string,o generateName:string,o namespace:string,o selfLink:string,o uid:string,o "
     "resourceVersion:string,o generation:int,o creationTimestamp:Time deletionTimestamp:*Time,o "
     "deletionGracePeriodSeconds:*int,o labels:map,o annotations:map,o ownerReferences:[]any,o "
     "finalizers:[]string,o clusterName:string,o managedFields:[]any,o")
_def("LabelSelector", "matchLabels:map,o matchExpressions:[]any,o")
_def("ObjectReference", "kind:string,o namespace:string,o name:string,o uid:string,o apiVersion:string,o "
     "resourceVersion:string,o fieldPath:string,o")
_def("LocalObjectReference", "name:string,o")

# -- core/v1 pod -------------------------------------------------------------
_def("PodTemplateSpec", "metadata:ObjectMeta,o spec:PodSpec,o")
_def("PodSpec", "volumes:[]Volume,o initContainers:[]Container,o containers:[]Container "
     "ephemeralContainers:[]any,o restartPolicy:string,o terminationGracePeriodSeconds:*int,o "
     "activeDeadlineSeconds:*int,o dnsPolicy:string,o nodeSelector:map,o serviceAccountName:string,o "
     "serviceAccount:string,o automountServiceAccountToken:*bool,o nodeName:string,o hostNetwork:bool,o "
     "hostPID:bool,o hostIPC:bool,o shareProcessNamespace:*bool,o securityContext:*PodSecurityContext,o "
     "imagePullSecrets:[]LocalObjectReference,o hostname:string,o subdomain:string,o affinity:*any,o "
     "schedulerName:string,o tolerations:[]any,o hostAliases:[]any,o priorityClassName:string,o "
     "priority:*int,o dnsConfig:*any,o readinessGates:[]any,o runtimeClassName:*string,o "
     "enableServiceLinks:*bool,o preemptionPolicy:*string,o overhead:map,o topologySpreadConstraints:[]any,o "
     "setHostnameAsFQDN:*bool,o")
_def("Container", "name:string image:string,o command:[]string,o args:[]string,o workingDir:string,o "
     "ports:[]ContainerPort,o envFrom:[]any,o env:[]EnvVar,o resources:ResourceRequirements,o "
     "volumeMounts:[]VolumeMount,o volumeDevices:[]any,o livenessProbe:*Probe,o readinessProbe:*Probe,o "
     "startupProbe:*Probe,o lifecycle:*any,o terminationMessagePath:string,o terminationMessagePolicy:string,o "
     "imagePullPolicy:string,o securityContext:*SecurityContext,o stdin:bool,o stdinOnce:bool,o tty:bool,o")
_def("ContainerPort", "name:string,o hostPort:int,o containerPort:int protocol:string,o hostIP:string,o")
_def("EnvVar", "name:string value:string,o valueFrom:*any,o")
_def("ResourceRequirements", "limits:map:Quantity,o requests:map:Quantity,o")
_def("VolumeMount", "name:string readOnly:bool,o mountPath:string subPath:string,o mountPropagation:*string,o "
     "subPathExpr:string,o")
_def("Volume", "name:string inline:VolumeSource")
_def("VolumeSource", "hostPath:*HostPathVolumeSource,o emptyDir:*EmptyDirVolumeSource,o gcePersistentDisk:*any,o "
     "awsElasticBlockStore:*any,o gitRepo:*any,o secret:*SecretVolumeSource,o nfs:*any,o iscsi:*any,o "
     "glusterfs:*any,o persistentVolumeClaim:*PersistentVolumeClaimVolumeSource,o rbd:*any,o flexVolume:*any,o "
     "cinder:*any,o cephfs:*any,o flocker:*any,o downwardAPI:*any,o fc:*any,o azureFile:*any,o "
     "configMap:*ConfigMapVolumeSource,o vsphereVolume:*any,o quobyte:*any,o azureDisk:*any,o "
     "photonPersistentDisk:*any,o projected:*any,o portworxVolume:*any,o scaleIO:*any,o storageos:*any,o "
     "csi:*any,o ephemeral:*any,o")
_def("HostPathVolumeSource", "path:string type:*string,o")
_def("EmptyDirVolumeSource", "medium:string,o sizeLimit:*Quantity,o")
_def("PersistentVolumeClaimVolumeSource", "claimName:string readOnly:bool,o")
_def("SecretVolumeSource", "secretName:string,o items:[]KeyToPath,o defaultMode:*int,o optional:*bool,o")
_def("ConfigMapVolumeSource", "name:string,o items:[]KeyToPath,o defaultMode:*int,o optional:*bool,o")
_def("KeyToPath", "key:string path:string mode:*int,o")
_def("SecurityContext", "capabilities:*Capabilities,o privileged:*bool,o seLinuxOptions:*any,o "
     "windowsOptions:*any,o runAsUser:*int,o runAsGroup:*int,o runAsNonRoot:*bool,o "
     "readOnlyRootFilesystem:*bool,o allowPrivilegeEscalation:*bool,o procMount:*string,o seccompProfile:*any,o")
_def("Capabilities", "add:[]string,o drop:[]string,o")
_def("PodSecurityContext", "seLinuxOptions:*any,o windowsOptions:*any,o runAsUser:*int,o runAsGroup:*int,o "
     "runAsNonRoot:*bool,o supplementalGroups:[]int,o fsGroup:*int,o sysctls:[]any,o "
     "fsGroupChangePolicy:*string,o seccompProfile:*any,o")
_def("Probe", "exec:*ExecAction,o httpGet:*any,o tcpSocket:*any,o initialDelaySeconds:int,o timeoutSeconds:int,o "
     "periodSeconds:int,o successThreshold:int,o failureThreshold:int,o")
_def("ExecAction", "command:[]string,o")
_def("PodStatus", "phase:string,o conditions:[]any,o message:string,o reason:string,o nominatedNodeName:string,o "
     "hostIP:string,o podIP:string,o podIPs:[]any,o startTime:*Time,o initContainerStatuses:[]any,o "
     "containerStatuses:[]any,o qosClass:string,o ephemeralContainerStatuses:[]any,o")

# -- workloads ------------------------------------------------------------------
_META = "inline:TypeMeta metadata:ObjectMeta,o "
_def("Pod", _META + "spec:PodSpec,o status:PodStatus,o")
_def("Deployment", _META + "spec:DeploymentSpec,o status:DeploymentStatus,o")
_def("DeploymentSpec", "replicas:*int,o selector:*LabelSelector template:PodTemplateSpec strategy:DeploymentStrategy,o "
     "minReadySeconds:int,o revisionHistoryLimit:*int,o paused:bool,o progressDeadlineSeconds:*int,o")
# extensions/v1beta1 and apps/v1beta1: selector is omitempty and rollbackTo exists
_def("DeploymentV1beta1", _META + "spec:DeploymentSpecV1beta1,o status:DeploymentStatus,o")
_def("DeploymentSpecV1beta1", "replicas:*int,o selector:*LabelSelector,o template:PodTemplateSpec "
     "strategy:DeploymentStrategy,o minReadySeconds:int,o revisionHistoryLimit:*int,o paused:bool,o "
     "rollbackTo:*any,o progressDeadlineSeconds:*int,o")
_def("DeploymentStrategy", "type:string,o rollingUpdate:*any,o")
_def("DeploymentStatus", "observedGeneration:int,o replicas:int,o updatedReplicas:int,o readyReplicas:int,o "
     "availableReplicas:int,o unavailableReplicas:int,o conditions:[]any,o collisionCount:*int,o")
_def("DaemonSet", _META + "spec:DaemonSetSpec,o status:DaemonSetStatus,o")
_def("DaemonSetSpec", "selector:*LabelSelector template:PodTemplateSpec updateStrategy:DaemonSetUpdateStrategy,o "
     "minReadySeconds:int,o revisionHistoryLimit:*int,o")
# extensions/v1beta1: selector is omitempty and templateGeneration exists
_def("DaemonSetV1beta1", _META + "spec:DaemonSetSpecV1beta1,o status:DaemonSetStatus,o")
_def("DaemonSetSpecV1beta1", "selector:*LabelSelector,o template:PodTemplateSpec "
     "updateStrategy:DaemonSetUpdateStrategy,o minReadySeconds:int,o templateGeneration:int,o "
     "revisionHistoryLimit:*int,o")
_def("DaemonSetUpdateStrategy", "type:string,o rollingUpdate:*any,o")
_def("DaemonSetStatus", "currentNumberScheduled:int numberMisscheduled:int desiredNumberScheduled:int numberReady:int "
     "observedGeneration:int,o updatedNumberScheduled:int,o numberAvailable:int,o numberUnavailable:int,o "
     "collisionCount:*int,o conditions:[]any,o")
_def("StatefulSet", _META + "spec:StatefulSetSpec,o status:StatefulSetStatus,o")
_def("StatefulSetSpec", "replicas:*int,o selector:*LabelSelector template:PodTemplateSpec "
     "volumeClaimTemplates:[]PersistentVolumeClaim,o serviceName:string podManagementPolicy:string,o "
     "updateStrategy:StatefulSetUpdateStrategy,o revisionHistoryLimit:*int,o")
_def("StatefulSetUpdateStrategy", "type:string,o rollingUpdate:*any,o")
_def("StatefulSetStatus", "observedGeneration:int,o replicas:int readyReplicas:int,o currentReplicas:int,o "
     "updatedReplicas:int,o currentRevision:string,o updateRevision:string,o collisionCount:*int,o "
     "conditions:[]any,o")
# apps/v1beta1: selector is omitempty, status.observedGeneration is a pointer
_def("StatefulSetV1beta1", _META + "spec:StatefulSetSpecV1beta1,o status:StatefulSetStatusV1beta1,o")
_def("StatefulSetSpecV1beta1", "replicas:*int,o selector:*LabelSelector,o template:PodTemplateSpec "
     "volumeClaimTemplates:[]PersistentVolumeClaim,o serviceName:string podManagementPolicy:string,o "
     "updateStrategy:StatefulSetUpdateStrategy,o revisionHistoryLimit:*int,o")
_def("StatefulSetStatusV1beta1", "observedGeneration:*int,o replicas:int readyReplicas:int,o currentReplicas:int,o "
     "updatedReplicas:int,o currentRevision:string,o updateRevision:string,o collisionCount:*int,o "
     "conditions:[]any,o")
_def("ReplicaSet", _META + "spec:ReplicaSetSpec,o status:ReplicaSetStatus,o")
_def("ReplicaSetSpec", "replicas:*int,o minReadySeconds:int,o selector:*LabelSelector template:PodTemplateSpec,o")
_def("ReplicaSetV1beta1", _META + "spec:ReplicaSetSpecV1beta1,o status:ReplicaSetStatus,o")
_def("ReplicaSetSpecV1beta1", "replicas:*int,o minReadySeconds:int,o selector:*LabelSelector,o "
     "template:PodTemplateSpec,o")
_def("ReplicaSetStatus", "replicas:int fullyLabeledReplicas:int,o readyReplicas:int,o availableReplicas:int,o "
     "observedGeneration:int,o conditions:[]any,o")
_def("CronJob", _META + "spec:CronJobSpec,o status:CronJobStatus,o")
_def("CronJobSpec", "schedule:string startingDeadlineSeconds:*int,o concurrencyPolicy:string,o suspend:*bool,o "
     "jobTemplate:JobTemplateSpec successfulJobsHistoryLimit:*int,o failedJobsHistoryLimit:*int,o")
_def("JobTemplateSpec", "metadata:ObjectMeta,o spec:JobSpec,o")
_def("CronJobStatus", "active:[]ObjectReference,o lastScheduleTime:*Time,o")
_def("HorizontalPodAutoscaler", _META + "spec:HPASpec,o status:HPAStatus,o")
_def("HPASpec", "scaleTargetRef:CrossVersionObjectReference minReplicas:*int,o maxReplicas:int "
     "targetCPUUtilizationPercentage:*int,o")
_def("HPAStatus", "observedGeneration:*int,o lastScaleTime:*Time,o currentReplicas:int desiredReplicas:int "
     "currentCPUUtilizationPercentage:*int,o")
_def("CrossVersionObjectReference", "kind:string name:string apiVersion:string,o")
# autoscaling/v2beta1 and v2beta2 share the object shape down to the metric sources
_def("HorizontalPodAutoscalerV2", _META + "spec:HPASpecV2,o status:HPAStatusV2,o")
_def("HPASpecV2", "scaleTargetRef:CrossVersionObjectReference minReplicas:*int,o maxReplicas:int "
     "metrics:[]any,o behavior:*any,o")
_def("HPAStatusV2", "observedGeneration:*int,o lastScaleTime:*Time,o currentReplicas:int desiredReplicas:int "
     "currentMetrics:[]any conditions:[]any")
_def("Job", _META + "spec:JobSpec,o status:JobStatus,o")
_def("JobSpec", "parallelism:*int,o completions:*int,o activeDeadlineSeconds:*int,o backoffLimit:*int,o "
     "selector:*LabelSelector,o manualSelector:*bool,o template:PodTemplateSpec ttlSecondsAfterFinished:*int,o")
_def("JobStatus", "conditions:[]any,o startTime:*Time,o completionTime:*Time,o active:int,o succeeded:int,o failed:int,o")
_def("ReplicationController", _META + "spec:ReplicationControllerSpec,o status:ReplicationControllerStatus,o")
_def("ReplicationControllerSpec", "replicas:*int,o minReadySeconds:int,o selector:map,o template:*PodTemplateSpec,o")
_def("ReplicationControllerStatus", "replicas:int fullyLabeledReplicas:int,o readyReplicas:int,o availableReplicas:int,o "
     "observedGeneration:int,o conditions:[]any,o")
_def("DeploymentConfig", _META + "spec:DeploymentConfigSpec status:DeploymentConfigStatus")
_def("DeploymentConfigSpec", "strategy:OpenShiftDeploymentStrategy minReadySeconds:int,o triggers:[]DeploymentTriggerPolicy "
     "replicas:int revisionHistoryLimit:*int,o test:bool paused:bool,o selector:map,o template:*PodTemplateSpec,o")
_def("OpenShiftDeploymentStrategy", "type:string,o customParams:*any,o recreateParams:*any,o rollingParams:*any,o "
     "resources:ResourceRequirements,o labels:map,o annotations:map,o activeDeadlineSeconds:*int,o")
_def("DeploymentTriggerPolicy", "type:string,o imageChangeParams:*DeploymentTriggerImageChangeParams,o")
_def("DeploymentTriggerImageChangeParams", "automatic:bool,o containerNames:[]string,o from:ObjectReference "
     "lastTriggeredImage:string,o")
_def("DeploymentConfigStatus", "latestVersion:int observedGeneration:int replicas:int updatedReplicas:int "
     "availableReplicas:int unavailableReplicas:int details:*any,o conditions:[]any,o readyReplicas:int,o")

# -- networking ---------------------------------------------------------------
_def("Service", _META + "spec:ServiceSpec,o status:ServiceStatus,o")
_def("ServiceSpec", "ports:[]ServicePort,o selector:map,o clusterIP:string,o type:string,o externalIPs:[]string,o "
     "sessionAffinity:string,o loadBalancerIP:string,o loadBalancerSourceRanges:[]string,o externalName:string,o "
     "externalTrafficPolicy:string,o healthCheckNodePort:int,o publishNotReadyAddresses:bool,o "
     "sessionAffinityConfig:*any,o ipFamily:*string,o topologyKeys:[]string,o")
_def("ServicePort", "name:string,o protocol:string,o appProtocol:*string,o port:int targetPort:IntOrString,o nodePort:int,o")
_def("ServiceStatus", "loadBalancer:LoadBalancerStatus,o")
_def("LoadBalancerStatus", "ingress:[]any,o")
_def("Ingress", _META + "spec:IngressSpec,o status:IngressStatus,o")
_def("IngressSpec", "ingressClassName:*string,o defaultBackend:*IngressBackend,o tls:[]IngressTLS,o rules:[]IngressRule,o")
_def("IngressBackend", "service:*IngressServiceBackend,o resource:*any,o")
_def("IngressServiceBackend", "name:string port:ServiceBackendPort,o")
_def("ServiceBackendPort", "name:string,o number:int,o")
_def("IngressRule", "host:string,o http:*HTTPIngressRuleValue,o")
_def("HTTPIngressRuleValue", "paths:[]HTTPIngressPath")
_def("HTTPIngressPath", "path:string,o pathType:*string,o backend:IngressBackend")
_def("IngressTLS", "hosts:[]string,o secretName:string,o")
_def("IngressStatus", "loadBalancer:LoadBalancerStatus,o")
_def("IngressV1beta1", _META + "spec:IngressSpecV1beta1,o status:IngressStatus,o")
_def("IngressSpecV1beta1", "ingressClassName:*string,o backend:*IngressBackendV1beta1,o tls:[]IngressTLS,o "
     "rules:[]IngressRuleV1beta1,o")
_def("IngressBackendV1beta1", "serviceName:string,o servicePort:IntOrString,o resource:*any,o")
_def("IngressRuleV1beta1", "host:string,o http:*HTTPIngressRuleValueV1beta1,o")
_def("HTTPIngressRuleValueV1beta1", "paths:[]HTTPIngressPathV1beta1")
_def("HTTPIngressPathV1beta1", "path:string,o pathType:*string,o backend:IngressBackendV1beta1")
_def("Route", _META + "spec:RouteSpec status:RouteStatus,o")
_def("RouteSpec", "host:string,o subdomain:string,o path:string,o to:RouteTargetReference alternateBackends:[]any,o "
     "port:*RoutePort,o tls:*any,o wildcardPolicy:string,o")
_def("RouteTargetReference", "kind:string name:string weight:*int")
_def("RoutePort", "targetPort:IntOrString")
_def("RouteStatus", "ingress:[]RouteIngress")
_def("RouteIngress", "host:string,o routerName:string,o conditions:[]any,o wildcardPolicy:string,o "
     "routerCanonicalHostname:string,o")
_def("NetworkPolicy", _META + "spec:NetworkPolicySpec,o")
_def("NetworkPolicySpec", "podSelector:LabelSelector ingress:[]NetworkPolicyIngressRule,o egress:[]any,o "
     "policyTypes:[]string,o")
_def("NetworkPolicyIngressRule", "ports:[]any,o from:[]NetworkPolicyPeer,o")
_def("NetworkPolicyPeer", "podSelector:*LabelSelector,o namespaceSelector:*LabelSelector,o ipBlock:*any,o")

# -- storage / config ------------------------------------------------------------
_def("ConfigMap", _META + "immutable:*bool,o data:map,o binaryData:map:bytes,o")
_def("Secret", _META + "immutable:*bool,o data:map:bytes,o stringData:map,o type:string,o")
_def("PersistentVolumeClaim", _META + "spec:PersistentVolumeClaimSpec,o status:PersistentVolumeClaimStatus,o")
_def("PersistentVolumeClaimSpec", "accessModes:[]string,o selector:*LabelSelector,o resources:ResourceRequirements,o "
     "volumeName:string,o storageClassName:*string,o volumeMode:*string,o dataSource:*any,o")
_def("PersistentVolumeClaimStatus", "phase:string,o accessModes:[]string,o capacity:map:Quantity,o conditions:[]any,o")
_def("ImageStream", _META + "spec:ImageStreamSpec status:ImageStreamStatus,o")
_def("ImageStreamSpec", "lookupPolicy:ImageLookupPolicy,o dockerImageRepository:string,o tags:[]TagReference,o")
_def("ImageLookupPolicy", "local:bool")
_def("TagReference", "name:string annotations:map from:*ObjectReference,o reference:bool,o generation:*int "
     "importPolicy:TagImportPolicy,o referencePolicy:TagReferencePolicy,o")
_def("TagImportPolicy", "insecure:bool,o scheduled:bool,o")
_def("TagReferencePolicy", "type:string")
_def("ImageStreamStatus", "dockerImageRepository:string publicDockerImageRepository:string,o tags:[]any,o")

# -- rbac ----------------------------------------------------------------------------
_def("Role", _META + "rules:[]PolicyRule")
_def("PolicyRule", "verbs:[]string apiGroups:[]string,o resources:[]string,o resourceNames:[]string,o "
     "nonResourceURLs:[]string,o")
_def("RoleBinding", _META + "subjects:[]Subject,o roleRef:RoleRef")
_def("Subject", "kind:string apiGroup:string,o name:string namespace:string,o")
_def("RoleRef", "apiGroup:string kind:string name:string")
_def("RoleBindingV1alpha1", _META + "subjects:[]SubjectV1alpha1,o roleRef:RoleRef")
_def("SubjectV1alpha1", "kind:string apiVersion:string,o name:string namespace:string,o")
# authorization.openshift.io/v1 (github.com/openshift/api/authorization/v1)
_def("RoleOpenShift", _META + "rules:[]PolicyRuleOpenShift")
_def("PolicyRuleOpenShift", "verbs:[]string attributeRestrictions:RawExtension apiGroups:[]string "
     "resources:[]string resourceNames:[]string,o nonResourceURLs:[]string,o")
_def("RoleBindingOpenShift", _META + "userNames:[]string groupNames:[]string subjects:[]ObjectReference "
     "roleRef:ObjectReference")
_def("ServiceAccount", _META + "secrets:[]ObjectReference,o imagePullSecrets:[]LocalObjectReference,o "
     "automountServiceAccountToken:*bool,o")

# -- knative -------------------------------------------------------------------------
_def("KnativeService", _META + "spec:KnativeServiceSpec,o status:KnativeServiceStatus,o")
_def("KnativeServiceSpec", "template:RevisionTemplateSpec,o traffic:[]any,o")
_def("RevisionTemplateSpec", "metadata:ObjectMeta,o spec:RevisionSpec,o")
_def("RevisionSpec", "inline:PodSpec containerConcurrency:*int,o timeoutSeconds:*int,o")
_def("KnativeServiceStatus", "observedGeneration:int,o conditions:[]any,o annotations:map,o "
     "latestReadyRevisionName:string,o latestCreatedRevisionName:string,o url:*any,o address:*any,o traffic:[]any,o")

# -- tekton ---------------------------------------------------------------------------
_def("Pipeline", _META + "spec:PipelineSpec")
_def("PipelineSpec", "description:string,o resources:[]any,o tasks:[]PipelineTask,o params:[]ParamSpec,o "
     "workspaces:[]PipelineWorkspaceDeclaration,o results:[]any,o finally:[]any,o")
_def("PipelineTask", "name:string,o taskRef:*TaskRef,o taskSpec:*any,o conditions:[]any,o when:[]any,o retries:int,o "
     "runAfter:[]string,o resources:*any,o params:[]Param,o workspaces:[]WorkspacePipelineTaskBinding,o timeout:*any,o")
_def("TaskRef", "name:string,o kind:string,o apiVersion:string,o bundle:string,o")
_def("Param", "name:string value:ArrayOrString")
_def("ParamSpec", "name:string type:string,o description:string,o default:*any,o")
_def("PipelineWorkspaceDeclaration", "name:string description:string,o optional:bool,o")
_def("WorkspacePipelineTaskBinding", "name:string workspace:string subPath:string,o")
_def("PipelineRun", _META + "spec:PipelineRunSpec,o status:PipelineRunStatus,o")
_def("PipelineRunSpec", "pipelineRef:*PipelineRef,o pipelineSpec:*any,o resources:[]any,o params:[]Param,o "
     "serviceAccountName:string,o serviceAccountNames:[]any,o status:string,o timeout:*any,o podTemplate:*any,o "
     "workspaces:[]WorkspaceBinding,o taskRunSpecs:[]any,o")
_def("PipelineRef", "name:string,o apiVersion:string,o bundle:string,o")
_def("WorkspaceBinding", "name:string subPath:string,o volumeClaimTemplate:*PersistentVolumeClaim,o "
     "persistentVolumeClaim:*any,o emptyDir:*any,o configMap:*any,o secret:*any,o")
_def("PipelineRunStatus", "observedGeneration:int,o conditions:[]any,o annotations:map,o podName:string,o "
     "startTime:*Time,o completionTime:*Time,o taskRuns:map,o runs:map,o pipelineResults:[]any,o "
     "pipelineSpec:*any,o skippedTasks:[]any,o")
_def("EventListener", _META + "spec:EventListenerSpec status:EventListenerStatus,o")
_def("EventListenerSpec", "serviceAccountName:string triggers:[]EventListenerTrigger serviceType:string,o "
     "replicas:*int,o podTemplate:ELPodTemplate,o namespaceSelector:ELNamespaceSelector,o resources:ELResources,o")
_def("ELPodTemplate", "tolerations:[]any,o nodeSelector:map,o")
_def("ELNamespaceSelector", "matchNames:[]string,o")
_def("ELResources", "kubernetesResource:*any,o")
_def("EventListenerTrigger", "bindings:[]EventListenerBinding template:*EventListenerTemplate,o triggerRef:string,o "
     "name:string,o interceptors:[]any,o serviceAccount:*any,o")
_def("EventListenerBinding", "name:string,o kind:string,o ref:string,o spec:*any,o apiversion:string,o")
_def("EventListenerTemplate", "name:string,o ref:*string,o apiversion:string,o")
_def("EventListenerStatus", "observedGeneration:int,o conditions:[]any,o annotations:map,o address:*any,o "
     "configuration:EventListenerConfig")
_def("EventListenerConfig", "generatedName:string")
_def("TriggerBinding", _META + "spec:TriggerBindingSpec status:EmptyStatus")
_def("TriggerBindingSpec", "params:[]any,o")
_def("EmptyStatus", "")
_def("TriggerTemplate", _META + "spec:TriggerTemplateSpec status:EmptyStatus")
_def("TriggerTemplateSpec", "params:[]ParamSpec,o resourcetemplates:[]RawExtension,o")


# (group/version, kind) -> struct type; "*" group wildcard per kind
KIND_TYPES = {
    "Pod": "Pod", "Deployment": "Deployment", "DaemonSet": "DaemonSet", "Job": "Job",
    "ReplicationController": "ReplicationController", "DeploymentConfig": "DeploymentConfig",
    "Service": "Service", "Ingress": "Ingress", "Route": "Route", "NetworkPolicy": "NetworkPolicy",
    "ConfigMap": "ConfigMap", "Secret": "Secret", "PersistentVolumeClaim": "PersistentVolumeClaim",
    "ImageStream": "ImageStream", "Role": "Role", "RoleBinding": "RoleBinding", "ServiceAccount": "ServiceAccount",
    "Pipeline": "Pipeline", "PipelineRun": "PipelineRun", "EventListener": "EventListener",
    "TriggerBinding": "TriggerBinding", "TriggerTemplate": "TriggerTemplate",
    "StatefulSet": "StatefulSet", "ReplicaSet": "ReplicaSet", "CronJob": "CronJob",
    "HorizontalPodAutoscaler": "HorizontalPodAutoscaler",
}


def type_for(obj):
    """Struct type used to marshal ``obj`` (None = pass-through)."""
    kind = obj.get("kind", "")
    gv = obj.get("apiVersion", "")
    if kind == "Service" and gv.startswith("serving.knative.dev/"):
        return "KnativeService"
    if kind == "Ingress" and gv in ("networking.k8s.io/v1beta1", "extensions/v1beta1"):
        return "IngressV1beta1"
    v = _VERSIONED.get((gv, kind))
    return v if v is not None else KIND_TYPES.get(kind)


# types whose fields differ between the versions a kind is registered under
_VERSIONED = {
    ("extensions/v1beta1", "Deployment"): "DeploymentV1beta1",
    ("apps/v1beta1", "Deployment"): "DeploymentV1beta1",
    ("extensions/v1beta1", "DaemonSet"): "DaemonSetV1beta1",
    ("extensions/v1beta1", "ReplicaSet"): "ReplicaSetV1beta1",
    ("apps/v1beta1", "StatefulSet"): "StatefulSetV1beta1",
    ("autoscaling/v2beta1", "HorizontalPodAutoscaler"): "HorizontalPodAutoscalerV2",
    ("autoscaling/v2beta2", "HorizontalPodAutoscaler"): "HorizontalPodAutoscalerV2",
    ("rbac.authorization.k8s.io/v1alpha1", "RoleBinding"): "RoleBindingV1alpha1",
    ("authorization.openshift.io/v1", "Role"): "RoleOpenShift",
    ("authorization.openshift.io/v1", "RoleBinding"): "RoleBindingOpenShift",
}


# -- typed-decode checks -------------------------------------------------------
# The reference decodes manifests with client-go's UniversalDeserializer:
# sigs.k8s.io/yaml turns the YAML into JSON (go-yaml v2 scalars) and
# encoding/json fills the typed struct, failing the whole object on a type
# mismatch (a quoted ``containerPort: "80"``, ``replicas: 1.5``, a label
# ``version: 1``).  :func:`check` reports the first such mismatch the same way,
# so these objects are skipped with a message instead of flowing on with
# values no Go field could hold.  Unknown fields are ignored (non-strict
# decoding); ``any``/``RawExtension``/untyped maps are not looked into.

_STRING_MAPS = {("ObjectMeta", "labels"), ("ObjectMeta", "annotations"), ("PodSpec", "nodeSelector"),
                ("LabelSelector", "matchLabels")}


def _json_kind(v):
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, (int, float)):
        return "number"
    if isinstance(v, str):
        return "string"
    if isinstance(v, list):
        return "array"
    if isinstance(v, dict):
        return "object"
    return "value"


def _mismatch(v, typ, path):
    raise ValueError("json: cannot unmarshal %s into Go struct field %s of type %s" % (_json_kind(v), path, typ))


def _check_value(v, typ, path):
    if v is None:
        return
    if typ.startswith("*"):
        return _check_value(v, typ[1:], path)
    if typ.startswith("[]"):
        if not isinstance(v, list):
            _mismatch(v, typ, path)
        for x in v:
            _check_value(x, typ[2:], path)
        return
    if typ == "map" or typ.startswith("map:"):
        if not isinstance(v, dict):
            _mismatch(v, typ, path)
        if typ.startswith("map:"):
            for x in v.values():
                _check_value(x, typ[4:], path)
        return
    if typ in ("string", "Time", "bytes"):
        if not isinstance(v, str):
            _mismatch(v, typ, path)
    elif typ == "int":
        if isinstance(v, bool) or not isinstance(v, (int, float)) or (isinstance(v, float) and not v.is_integer()):
            _mismatch(v, typ, path)
    elif typ == "bool":
        if not isinstance(v, bool):
            _mismatch(v, typ, path)
    elif typ == "IntOrString":
        if isinstance(v, bool) or not isinstance(v, (int, float, str)) or (isinstance(v, float) and not v.is_integer()):
            _mismatch(v, typ, path)
    elif typ == "Quantity":
        if isinstance(v, bool) or not isinstance(v, (int, float, str)):
            _mismatch(v, typ, path)
    elif typ in _STRUCTS:
        _check_struct(v, typ, path)


def _check_struct(d, typ, path):
    if not isinstance(d, dict):
        _mismatch(d, typ, path)
    for jname, ftype, _omit in _fields(typ):
        if jname == "inline":
            _check_struct(d, ftype, path)
            continue
        v = d.get(jname)
        if v is None:
            continue
        fpath = "%s.%s" % (path, jname) if path else jname
        if (typ, jname) in _STRING_MAPS:
            if not isinstance(v, dict):
                _mismatch(v, "map[string]string", typ + "." + fpath)
            for x in v.values():
                if x is not None and not isinstance(x, str):
                    _mismatch(x, "string", typ + "." + fpath)
            continue
        _check_value(v, ftype, fpath)


def check(obj):
    """Raise ValueError if ``obj`` could not be decoded into its Go type."""
    typ = type_for(obj)
    if typ is None:
        md = obj.get("metadata")
        if md is not None:
            _check_struct(md, "ObjectMeta", "metadata")
        return
    _check_struct(obj, typ, "")


def _is_empty(v, typ):
    if v is None:
        return True
    if typ.startswith("*"):
        return False
    if typ in ("string",):
        return v == ""
    if typ == "int":
        return v == 0
    if typ == "bool":
        return v is False
    if typ.startswith("[]") or typ.startswith("map") or typ == "bytes":
        return len(v) == 0
    if typ == "any":
        return isinstance(v, (dict, list, str)) and len(v) == 0 or v is False or v == 0
    return False


def _zero(typ):
    if typ == "string":
        return ""
    if typ == "int":
        return 0
    if typ == "bool":
        return False
    if typ == "Time":
        return None
    if typ == "IntOrString":
        return 0
    if typ in ("ArrayOrString",):
        return ""
    if typ in _STRUCTS:
        return _marshal_struct({}, typ)
    return None


def _marshal_value(v, typ):
    if typ.startswith("*"):
        return None if v is None else _marshal_value(v, typ[1:])
    if typ.startswith("[]"):
        if v is None:
            return None
        return [_marshal_value(x, typ[2:]) for x in v]
    if typ == "map":
        return None if v is None else dict(v)
    if typ.startswith("map:"):
        if v is None:
            return None
        return {k: _marshal_value(x, typ[4:]) for k, x in v.items()}
    if typ == "bytes":
        if v is None:
            return None
        if isinstance(v, str):
            return v
        import base64
        return base64.b64encode(bytes(v)).decode()
    if typ == "Time":
        return v if v else None
    if typ in ("string", "Quantity", "ArrayOrString"):
        return v if isinstance(v, str) else ("" if v is None else v)
    if typ == "int":
        return v
    if typ == "bool":
        return bool(v)
    if typ == "IntOrString":
        return v
    if typ == "any":
        return v
    if typ == "RawExtension":
        return marshal(v) if isinstance(v, dict) else v
    if typ in _STRUCTS:
        return _marshal_struct(v or {}, typ)
    return v


_SKIP = object()
_EMPTY_STRUCT = object()
_plans = {}
_empty = {}


def _plan(typ):
    """Per struct type: (json name, field type, omitempty, value when absent,
    compiled value marshaller, compiled omitempty test)."""
    pl = _plans.get(typ)
    if pl is None:
        pl = []
        for jname, ftype, omit in _fields(typ):
            if jname == "inline":
                absent = None
            elif ftype in _STRUCTS:
                absent = _EMPTY_STRUCT
            elif ftype == "Time":
                absent = None
            elif omit:
                absent = _SKIP
            elif ftype.startswith("*") or ftype.startswith("[]") or ftype.startswith("map") or ftype in ("any", "bytes"):
                absent = None
            else:
                absent = _zero(ftype)
            empty = _empty_fn(ftype) if omit else None
            pl.append((jname, ftype, omit, absent, _value_fn(ftype), empty))
        pl = _plans[typ] = tuple(pl)
    return pl


# -- compiled per-type marshallers (same semantics as _marshal_value/_is_empty,
#    without re-parsing the type string for every value) ----------------------

_value_fns = {}
_empty_fns = {}


def _ident(v):
    return v


def _str_value(v):
    return v if isinstance(v, str) else ("" if v is None else v)


def _value_fn(typ):
    fn = _value_fns.get(typ)
    if fn is None:
        fn = _value_fns[typ] = _compile_value(typ)
    return fn


def _compile_value(typ):
    if typ.startswith("*"):
        inner = _value_fn(typ[1:])
        return lambda v: None if v is None else inner(v)
    if typ.startswith("[]"):
        inner = _value_fn(typ[2:])
        return lambda v: None if v is None else [inner(x) for x in v]
    if typ == "map":
        return lambda v: None if v is None else dict(v)
    if typ.startswith("map:"):
        inner = _value_fn(typ[4:])
        return lambda v: None if v is None else {k: inner(x) for k, x in v.items()}
    if typ in ("bytes", "Time", "RawExtension"):
        return lambda v: _marshal_value(v, typ)
    if typ in ("string", "Quantity", "ArrayOrString"):
        return _str_value
    if typ == "bool":
        return bool
    if typ in _STRUCTS:
        return lambda v: _marshal_struct(v or {}, typ)
    return _ident  # int, IntOrString, any, unknown


def _empty_fn(typ):
    fn = _empty_fns.get(typ)
    if fn is None:
        if typ.startswith("*"):
            fn = lambda v: False  # noqa: E731
        elif typ == "string":
            fn = lambda v: v == ""  # noqa: E731
        elif typ == "int":
            fn = lambda v: v == 0  # noqa: E731
        elif typ == "bool":
            fn = lambda v: v is False  # noqa: E731
        elif typ.startswith("[]") or typ.startswith("map") or typ == "bytes":
            fn = lambda v: len(v) == 0  # noqa: E731
        else:
            fn = lambda v, t=typ: _is_empty(v, t)  # noqa: E731
        _empty_fns[typ] = fn
    return fn


def _empty_struct(typ):
    # shared and read-only: marshal output only feeds the serializer
    e = _empty.get(typ)
    if e is None:
        e = _empty[typ] = _marshal_fields({}, typ)
    return e


def _marshal_struct(d, typ):
    if not d:
        return _empty_struct(typ)
    return _marshal_fields(d, typ)


_keyed = {}


def _keyed_plan(typ):
    """(json name -> (omitempty, value fn, empty fn), inline struct types,
    {json name: value} of the fields an absent key still produces)."""
    kp = _keyed.get(typ)
    if kp is None:
        fields, inlines, base = {}, [], {}
        for jname, ftype, omit, absent, value, empty in _plan(typ):
            if jname == "inline":
                inlines.append(ftype)
                continue
            fields[jname] = (omit, value, empty)
            if absent is not _SKIP:
                base[jname] = _empty_struct(ftype) if absent is _EMPTY_STRUCT else absent
        kp = _keyed[typ] = (fields, tuple(inlines), base)
    return kp


def _marshal_fields(d, typ):
    # Driven by the keys present in ``d`` rather than by every field of the
    # struct (a PodSpec has ~40, a typical one sets 3): fields an absent key
    # still produces start from a per-type template.  Key order differs from
    # Go's struct order, which is fine: the only consumer (dumps_k8s) emits
    # every mapping sorted, as go-yaml does for the reference's Go maps.
    fields, inlines, base = _keyed_plan(typ)
    out = dict(base)
    for ftype in inlines:
        out.update(_marshal_struct(d, ftype))
    get = fields.get
    for k, v in d.items():
        f = get(k)
        if f is None or v is None:
            continue
        omit, value, empty = f
        if omit and empty(v):
            out.pop(k, None)
            continue
        out[k] = value(v)
    return out


_native_fn = None
_native_lock = _thread.RLock()


def _native_marshal():
    """``schema_marshal`` of the native extension (ops/csrc/k8s_marshal.cpp),
    compiled from the ``_STRUCTS`` field strings on first use; False when it is unavailable or
    ``M2K_NATIVE_MARSHAL=0``.  This module stays its specification."""
    global _native_fn
    if _native_fn is not None:
        return _native_fn
    with _native_lock:   # threads asking at once wait for one initialisation
        if _native_fn is None:
            fn = False
            import os
            try:
                if os.environ.get("M2K_NATIVE_MARSHAL", "1") != "0":
                    from ..ops import native
                    m = native.module()
                    if m is not None and hasattr(m, "schema_marshal"):
                        m.schema_init(_STRUCTS, _marshal_value)
                        fn = m.schema_marshal
            finally:
                _native_fn = fn
    return _native_fn


def _struct(d, typ):
    fn = _native_marshal()
    return fn(d, typ) if fn else _marshal_struct(d, typ)


def marshal(obj):
    """Go json.Marshal of a typed Kubernetes object given as a JSON-shaped dict."""
    typ = type_for(obj)
    if typ is None:
        out = dict(obj)
        md = out.get("metadata")
        if isinstance(md, dict):
            out["metadata"] = _struct(md, "ObjectMeta")
        elif "metadata" not in out:
            out["metadata"] = _struct({}, "ObjectMeta")
        return out
    return _struct(obj, typ)


def marshal_as(d, typ):
    return _struct(d, typ)

// Volumes web app frontend (reference crud-web-apps/volumes/frontend): PVC table (common resource
// table, polled) with the notebooks using each claim, create / delete, volume details (overview with
// the pods mounting it and conditions / events / YAML) and the PVCViewer (file browser) lifecycle: browse
// -> viewer created -> open its URL when ready -> close.
// `VWA` holds the pure parts (columns, viewer button state, request body) for the node tests.
(function (global) {
  "use strict";
  const kf = global.kf || (typeof require !== "undefined" ? require("../../../crud_backend/static/kf.js") : null);

  const VWA = {
    // confirm dialogs (services/actions.service.ts, index-default.component.ts)
    dialogs: {
      delete: (name) => ({ title: `Are you sure you want to delete this volume? ${name}`,
                           message: "Warning: All data in this volume will be lost.", accept: "DELETE",
                           confirmColor: "warn", cancel: "CANCEL", error: "", applying: "DELETING", width: "600px" }),
      closeViewer: (name) => ({ title: `Are you sure you want to close this viewer? ${name}`,
                                message: "Warning: Any running processes will terminate.", accept: "CLOSE",
                                confirmColor: "warn", cancel: "CANCEL", error: "", applying: "CLOSING", width: "600px" }),
    },
    columns(allNamespaces) {
      const cols = [
        { title: "Status", value: (r) => r.status.phase, html: (r) => kf.statusIcon(r.status) },
        { title: "Name", value: (r) => r.name, html: (r) => kf.nameLink(r) },
      ];
      if (allNamespaces) cols.push({ title: "Namespace", value: (r) => r.namespace });
      cols.push(
        { title: "Created at", kind: "date", value: (r) => r.age },
        { title: "Size", kind: "memory", value: (r) => r.capacity },
        { title: "Access Mode", value: (r) => (r.modes || []).join(", ") },
        { title: "Storage Class", value: (r) => r.class || "" },
        { title: "Used by", value: (r) => (r.notebooks || []).join(", "), sortable: false },
      );
      return cols;
    },
    // backend rows carry viewer {status, url} (volumes backend get.py); older payloads a bare status
    viewerState(row) {
      const v = row.viewer;
      return typeof v === "string" ? { status: v, url: null } : { status: (v || {}).status || "uninitialized", url: (v || {}).url || null };
    },
    browseLabel(row) {
      const v = VWA.viewerState(row);
      return v.status === "ready" ? "Open browser" : v.status === "uninitialized" ? "Browse" : `Browser ${v.status}`;
    },
    // Button states of index-default.component.ts parseIncomingData. `waiting` is the set of claims
    // whose viewer the user asked for; their window opens (autoOpen) once the viewer is ready.
    actionStates(row, waiting) {
      const v = VWA.viewerState(row), phase = row.status.phase;
      const deleteAction = (row.notebooks || []).length ? "unavailable" : phase === "terminating" ? "terminating" : "ready";
      // a claim that is only waiting for its first consumer may get the viewer as that consumer
      const firstConsumer = phase === "unavailable" && row.status.state === "WaitForFirstConsumer";
      let openAction = v.status, autoOpen = false;
      if (phase !== "ready" && !firstConsumer) openAction = "unavailable";
      else if (waiting && waiting.has(row.name)) {
        if (v.status === "ready") { autoOpen = true; waiting.delete(row.name); }
        else if (v.status === "uninitialized" || v.status === "waiting") openAction = "waiting";
      }
      const closeAction = v.status === "uninitialized" ? "unavailable" : v.status === "terminating" ? "waiting" : "ready";
      return { deleteAction, openAction, closeAction, autoOpen };
    },
    // volume-details-page/overview: the PVC's facts ("null" where unset, as the component shows),
    // owner chips, and the pods mounting it grouped into Notebooks / InferenceService links
    overview(pvc) {
      const spec = (pvc || {}).spec || {}, st = (pvc || {}).status || {};
      const owners = ((pvc || {}).metadata || {}).ownerReferences || [];
      return {
        accessModes: (st.accessModes || spec.accessModes || []).filter(Boolean),
        size: (st.capacity || {}).storage || ((spec.resources || {}).requests || {}).storage || "null",
        storageClass: spec.storageClassName || "null", volumeMode: spec.volumeMode || "null",
        volumeName: spec.volumeName || "null", ownerRefs: owners.map((r) => `${r.kind}: ${r.name}`),
      };
    },
    podGroups(pods, viewerUrl) {
      const groups = [];
      (pods || []).forEach((pod) => {
        const labels = (pod.metadata || {}).labels || {}, ns = (pod.metadata || {}).namespace;
        let name, group, url;
        if ("serving.kubeflow.org/inferenceservice" in labels) {
          const svc = labels["serving.kubeflow.org/inferenceservice"];
          name = `${svc} (${labels.component})`;
          group = "InferenceService";
          url = `${viewerUrl || ""}/models/details/${ns}/${svc}/`;
        } else if ("notebook-name" in labels) {
          name = labels["notebook-name"];
          group = "Notebooks";
          url = `${viewerUrl || ""}/jupyter/notebook/details/${ns}/${name}/`;
        } else return;
        let g = groups.find((x) => x.name === group);
        if (!g) groups.push(g = { name: group, links: [] });
        g.links.push({ name, url });
      });
      return groups;
    },
    podsMountedMessage(error) {
      return error ? `Failed to fetch mounted pods with error: ${error}` : "No pods are using this PVC.";
    },
    newPvcBody(name, size, mode, storageClass) {
      return { name, size: /[A-Za-z]$/.test(String(size)) ? String(size) : `${size}Gi`, mode, class: storageClass || "{empty}", type: "empty" };
    },
    validate(name, size) {
      const errs = [];
      const n = kf.validators.name(name);
      if (n) errs.push(n);
      if (kf.validators.memory(/[A-Za-z]$/.test(String(size)) ? size : `${size}Gi`)) errs.push(`Invalid size: ${size}`);
      return errs;
    },
  };

  function app() {
    const $ = (id) => document.getElementById(id);
    let poller = null, table = null, rows = [];
    const waiting = new Set();
    const openViewer = (r) => window.open(VWA.viewerState(r).url, `${r.name}: Volumes Viewer`, "height=600,width=800");
    async function namespaces() {
      let list = [];
      try { list = (await kf.call("GET", "/api/namespaces")).namespaces; } catch (e) { list = kf.namespace() ? [kf.namespace()] : []; }
      $("ns").innerHTML = list.map((n) => `<option value="${kf.esc(n)}">${kf.esc(n)}</option>`).join("");
      if (!kf.namespace() && list.length) kf.setNamespace(list[0]);
      $("ns").value = kf.namespace();
      $("ns").onchange = () => kf.setNamespace($("ns").value);
    }
    async function act(method, path, body) {
      try { await kf.call(method, path, body); } catch (e) { kf.snack(e.message, "ERROR"); }
      poller.reset();
    }
    const spec_has = (pvc, k) => !!((pvc || {}).spec || {})[k];
    // volume page: overview (+ pods mounted, conditions) / events / YAML (VWA pages/volume-details-page)
    function showDetails(ns, name) {
      const base = `/api/namespaces/${ns}/pvcs/${name}`;
      const e = kf.esc;
      return kf.details(`Volume ${ns}/${name}`, [
        { name: "Overview", render: async () => {
          const pvc = (await kf.call("GET", base)).pvc;
          const st = pvc.status || {};
          const ov = VWA.overview(pvc);
          let pods = [], err = "";
          try { pods = (await kf.call("GET", `${base}/pods`)).pods; } catch (x) { err = x.message; }
          const groups = VWA.podGroups(pods, "");
          const chips = (xs) => xs.map((x) => `<span class="chip">${e(x)}</span>`).join(" ");
          const rows = [["Name", pvc.metadata.name], ["Namespace", pvc.metadata.namespace], ["Created", pvc.metadata.creationTimestamp],
            ["Phase", st.phase || "-"], ["Size", ov.size], ["Storage class", ov.storageClass], ["Volume mode", ov.volumeMode]];
          if (spec_has(pvc, "volumeName")) rows.push(["Volume name", ov.volumeName]);
          return kf.kvTable(rows) +
            `<table class="kv"><tr><th>Access modes</th><td>${chips(ov.accessModes)}</td></tr>` +
            (ov.ownerRefs.length ? `<tr><th title="The PVC is deleted with the objects that own it">Owned by</th><td>${chips(ov.ownerRefs)}</td></tr>` : "") +
            "</table><h3>Pods Mounted</h3>" +
            (groups.length ? groups.map((g) => `<div class="vol-group"><b>${e(g.name)}</b> ` +
              g.links.map((l) => `<a class="pod-link" href="${e(l.url)}">${e(l.name)}</a>`).join(" ") + "</div>").join("")
              : `<p class="muted">${e(VWA.podsMountedMessage(err))}</p>`) +
            `<h3>Conditions</h3>${kf.conditionsTable(st.conditions)}`;
        } },
        { name: "Events", render: async () => kf.eventsTable((await kf.call("GET", `${base}/events`)).events) },
        { name: "YAML", render: async () => kf.yamlHtml(kf.toYaml((await kf.call("GET", base)).pvc)) },
      ]);
    }
    function tableConfig() {
      return {
        columns: VWA.columns(false), empty: "No volumes in this namespace.",
        actions: [
          { name: "browse", label: (r) => (r.openAction === "waiting" ? "Starting browser" : VWA.browseLabel(r)),
            enabled: (r) => ["ready", "uninitialized"].includes(r.openAction) },
          { name: "close", label: "Close browser", enabled: (r) => r.closeAction === "ready" },
          { name: "delete", label: "Delete", enabled: (r) => r.deleteAction === "ready" },
        ],
        onOpen: (r) => (r.status.phase === "terminating" ? kf.snack("PVC is unavailable now.", "WARNING") : showDetails(r.namespace, r.name)),
        onAction: (name, r) => {
          const ns = r.namespace, v = VWA.viewerState(r);
          if (name === "browse") {
            if (v.status === "ready" && v.url) openViewer(r);
            else if (v.status === "uninitialized") {
              waiting.add(r.name); r.openAction = "waiting"; table.setRows(rows);
              kf.call("POST", `/api/namespaces/${ns}/viewers`, { name: r.name })
                .catch((e) => { waiting.delete(r.name); kf.snack(e.message, "ERROR"); }).then(() => poller.reset());
            }
          }
          if (name === "close")
            kf.confirmDialog(VWA.dialogs.closeViewer(r.name), () => kf.call("DELETE", `/api/namespaces/${ns}/viewers/${r.name}`)).then((resp) => {
              if (resp === "accept") { waiting.delete(r.name); r.closeAction = "waiting"; table.setRows(rows); }
              poller.reset();
            });
          if (name === "delete")
            kf.confirmDialog(VWA.dialogs.delete(r.name), () => kf.call("DELETE", `/api/namespaces/${ns}/pvcs/${r.name}`)).then((resp) => {
              if (resp === "accept") {
                r.status = Object.assign({}, r.status, { phase: "terminating", message: "Preparing to delete the Volume..." });
                r.deleteAction = "unavailable"; waiting.delete(r.name); table.setRows(rows);
              }
              poller.reset();
            });
        },
      };
    }
    async function refresh() {
      const ns = kf.namespace();
      if (!ns) return null;
      const { pvcs } = await kf.call("GET", `/api/namespaces/${ns}/pvcs`);
      rows = pvcs.map((p) => {
        const r = Object.assign({ namespace: ns }, p), st = VWA.actionStates(r, waiting);
        if (st.autoOpen) openViewer(r);
        return Object.assign(r, st);
      });
      table.setRows(rows);
      return pvcs.map((p) => [p.name, p.status.phase, VWA.viewerState(p).status]);
    }
    async function open() {
      let classes = [], def = "";
      try { classes = (await kf.call("GET", "/api/storageclasses")).storageClasses; def = (await kf.call("GET", "/api/storageclasses/default")).defaultStorageClass; } catch (e) { /* not cluster-readable */ }
      $("f-class").innerHTML = `<option value="{empty}">(default${def ? ": " + kf.esc(def) : ""})</option><option value="{none}">(none)</option>` +
        classes.map((c) => `<option>${kf.esc(c)}</option>`).join("");
      $("f-error").textContent = "";
      $("dlg").showModal();
    }
    async function submit(ev) {
      if (ev.submitter && ev.submitter.value !== "ok") return;
      ev.preventDefault();
      const ns = kf.namespace();
      const errs = VWA.validate($("f-name").value, $("f-size").value);
      if (errs.length) { $("f-error").textContent = errs.join("; "); return; }
      try {
        await kf.call("POST", `/api/namespaces/${ns}/pvcs`, VWA.newPvcBody($("f-name").value, $("f-size").value, $("f-mode").value, $("f-class").value));
        $("dlg").close(); kf.snack(`Volume ${$("f-name").value} created`, "SUCCESS"); poller.reset();
      } catch (e) { $("f-error").textContent = e.message; }
    }
    (async function main() {
      poller = new kf.Poller(refresh);
      table = new kf.ResourceTable($("rows"), tableConfig());
      $("filter").oninput = (ev) => table.setFilter(ev.target.value);
      await namespaces();
      $("new").onclick = open;
      $("form").addEventListener("submit", submit);
      kf.onNamespace((ns) => { $("ns").value = ns; poller.reset(); });
      poller.start();
    })();
  }

  global.VWA = VWA;
  if (typeof module !== "undefined" && module.exports) module.exports = VWA;
  else if (typeof document !== "undefined") app();
})(typeof window !== "undefined" ? window : globalThis);
